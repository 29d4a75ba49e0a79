// Broker sets for BrokerSetAwareGoal: which set every broker is in and which set every replica belongs to.
//
//   BrokerSetResolutionHelper                config/BrokerSetResolutionHelper.java:25-60 (set id -> brokers, broker -> set)
//   NoOpBrokerSetAssignmentPolicy            config/NoOpBrokerSetAssignmentPolicy.java:70-86 (unresolved -> "unmapped")
//   TopicNameHashBrokerSetMappingPolicy      config/TopicNameHashBrokerSetMappingPolicy.java:30-70
//   ReplicaToOriginalBrokerSetMappingPolicy  config/ReplicaToOriginalBrokerSetMappingPolicy.java:20-26
//
// Set indices are ranks of the set ids in String order (the order TopicNameHashBrokerSetMappingPolicy sorts them in),
// so the consistent-hash bucket of a topic is directly its set index. The topic hash is Guava's (pinned version of the
// reference build, not vendored in the reference tree): Hashing.murmur3_128() over the UTF-8 bytes of the name,
// HashCode.asInt() (the low 32 bits of h1), Math.abs, then Hashing.consistentHash with its 64-bit LCG.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <climits>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "ccmi.h"

namespace ccmi {

namespace bsets {

inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

// MurmurHash3_x64_128 with seed 0; returns h1 (HashCode.asInt() reads its low 4 bytes, little-endian)
inline uint64_t murmur3x64h1(const uint8_t* d, size_t n) {
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  uint64_t h1 = 0, h2 = 0;
  const size_t blocks = n / 16;
  auto le64 = [](const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return v;
  };
  for (size_t i = 0; i < blocks; ++i) {
    uint64_t k1 = le64(d + 16 * i), k2 = le64(d + 16 * i + 8);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
  }
  const uint8_t* t = d + 16 * blocks;
  const size_t rem = n & 15;
  uint64_t k1 = 0, k2 = 0;
  for (size_t i = rem; i > 8; --i) k2 ^= (uint64_t)t[i - 1] << (8 * (i - 9));
  if (rem > 8) { k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2; }
  for (size_t i = std::min<size_t>(rem, 8); i > 0; --i) k1 ^= (uint64_t)t[i - 1] << (8 * (i - 1));
  if (rem > 0) { k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1; }
  h1 ^= n;
  h2 ^= n;
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  h1 += h2;
  return h1;
}

// Hashing.consistentHash(long, int): (int) of a double is Java's saturating narrowing
inline int32_t consistentHash(int64_t input, int32_t buckets) {
  uint64_t state = (uint64_t)input;
  int32_t candidate = 0;
  for (;;) {
    state = 2862933555777941757ULL * state + 1;
    const double next = (double)((int32_t)(state >> 33) + 1) / 2147483648.0;
    const double q = (double)(candidate + 1) / next;
    const int32_t n = q >= 2147483647.0 ? INT32_MAX : (int32_t)q;
    if (n >= 0 && n < buckets) candidate = n;
    else return candidate;
  }
}

inline int32_t topicBrokerSet(const std::string& topic, int32_t numSets) {
  if (numSets < 1) return -1;
  const int32_t h = (int32_t)(uint32_t)murmur3x64h1((const uint8_t*)topic.data(), topic.size());
  const int32_t a = h == INT32_MIN ? h : (h < 0 ? -h : h);  // Math.abs
  return consistentHash((int64_t)a, numSets);
}

}  // namespace bsets

// The resolved broker sets of one optimization call.
struct BrokerSets {
  int32_t numSets = 0;
  int32_t policy = CCMI_BROKER_SET_TOPIC_NAME_HASH;
  std::vector<std::string> names;  // String order
  std::vector<int32_t> ofBroker;   // [B] set index of every broker (dense index)

  // brokerIds: Kafka id of every dense broker index
  void resolve(const ccmi_balancing_constraint* c, const std::vector<int32_t>& brokerIds) {
    numSets = 0;
    names.clear();
    ofBroker.assign(brokerIds.size(), -1);
    if (!c || c->num_broker_sets <= 0) return;
    if (!c->broker_set_names || !c->broker_set_offset || (!c->broker_set_members && c->broker_set_offset[c->num_broker_sets] > 0))
      throw std::invalid_argument("broker set data without names / members");
    policy = c->broker_set_policy;
    if (policy != CCMI_BROKER_SET_TOPIC_NAME_HASH && policy != CCMI_BROKER_SET_ORIGINAL_BROKER)
      throw std::invalid_argument("unknown replica-to-broker-set mapping policy");
    // broker set id -> the session's broker ids. The session's ids are dense (ccmi_cluster_desc.broker_id[b] == b;
    // the builder numbers brokers in ascending Kafka-id order, ccmi_builder_broker_ids), so the caller maps its Kafka
    // ids through that table and passes -1 for an id the model does not hold; such a member (any id outside [0, B))
    // resolves to no broker, as a broker-set entry naming a broker absent from the cluster does in the reference.
    std::map<std::string, std::vector<int32_t>> byName;
    for (int s = 0; s < c->num_broker_sets; ++s) {
      auto& v = byName[c->broker_set_names[s]];
      for (int k = c->broker_set_offset[s]; k < c->broker_set_offset[s + 1]; ++k) v.push_back(c->broker_set_members[k]);
    }
    std::map<int32_t, int32_t> denseOf;
    for (size_t b = 0; b < brokerIds.size(); ++b) denseOf[brokerIds[b]] = (int32_t)b;
    std::vector<uint8_t> mapped(brokerIds.size(), 0);
    for (const auto& kv : byName)
      for (int32_t id : kv.second) {
        auto it = denseOf.find(id);
        if (it != denseOf.end()) mapped[it->second] = 1;
      }
    bool anyUnmapped = false;
    for (uint8_t m : mapped) anyUnmapped |= m == 0;
    if (anyUnmapped) {  // NoOpBrokerSetAssignmentPolicy: every unresolved broker joins "unmapped"
      auto& v = byName["unmapped"];
      for (size_t b = 0; b < brokerIds.size(); ++b)
        if (!mapped[b]) v.push_back(brokerIds[b]);
    }
    for (const auto& kv : byName) {  // std::map iterates in String (byte) order = Collections.sort for ASCII ids
      const int32_t idx = (int32_t)names.size();
      names.push_back(kv.first);
      for (int32_t id : kv.second) {
        auto it = denseOf.find(id);
        if (it != denseOf.end()) ofBroker[it->second] = idx;
      }
    }
    numSets = (int32_t)names.size();
  }
};

}  // namespace ccmi
