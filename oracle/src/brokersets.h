// ORACLE — test infrastructure only (see jsem.h header).
// Broker-set resolution for BrokerSetAwareGoal, restated from the reference and its Guava dependency:
//   TopicNameHashBrokerSetMappingPolicy.brokerSetIdForTopic   config/TopicNameHashBrokerSetMappingPolicy.java:60-70
//     Math.abs(Hashing.murmur3_128().hashString(topic, UTF_8).asInt()), then
//     sortedBrokerSetIds.get(Hashing.consistentHash(hash, sortedBrokerSetIds.size()))
//   Guava (com.google.guava, the reference build's dependency, not vendored): Murmur3_128HashFunction (x64 variant,
//   seed 0, HashCode bytes = h1 then h2 little-endian, asInt = first four bytes) and Hashing.consistentHash (64-bit
//   LCG 2862933555777941757 * s + 1, nextDouble = ((int)(s >>> 33) + 1) / 2^31). Pinned by the expected mappings of
//   TopicNameHashBrokerSetMappingPolicyTest.java:81-85,121-125.
#pragma once
#include <cstdint>
#include <cstring>
#include <string>

namespace oracle {

inline int32_t guavaMurmur3AsInt(const std::string& s) {
  const unsigned char* p = reinterpret_cast<const unsigned char*>(s.data());
  const size_t len = s.size();
  const uint64_t C1 = 0x87c37b91114253d5ULL, C2 = 0x4cf5ad432745937fULL;
  auto rotl = [](uint64_t x, int r) { return (x << r) | (x >> (64 - r)); };
  auto mixK1 = [&](uint64_t k) { k *= C1; k = rotl(k, 31); k *= C2; return k; };
  auto mixK2 = [&](uint64_t k) { k *= C2; k = rotl(k, 33); k *= C1; return k; };
  auto fmix = [](uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33;
    return k;
  };
  uint64_t h1 = 0, h2 = 0;
  size_t i = 0;
  for (; i + 16 <= len; i += 16) {  // Murmur3_128Hasher.process (little-endian longs)
    uint64_t k1 = 0, k2 = 0;
    for (int b = 0; b < 8; ++b) {
      k1 |= (uint64_t)p[i + b] << (8 * b);
      k2 |= (uint64_t)p[i + 8 + b] << (8 * b);
    }
    h1 ^= mixK1(k1);
    h1 = rotl(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    h2 ^= mixK2(k2);
    h2 = rotl(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
  }
  uint64_t k1 = 0, k2 = 0;  // processRemaining
  const size_t rem = len - i;
  for (size_t b = 0; b < rem; ++b) {
    if (b < 8) k1 ^= (uint64_t)p[i + b] << (8 * b);
    else k2 ^= (uint64_t)p[i + b] << (8 * (b - 8));
  }
  if (rem > 8) h2 ^= mixK2(k2);
  if (rem > 0) h1 ^= mixK1(k1);
  h1 ^= (uint64_t)len;  // makeHash
  h2 ^= (uint64_t)len;
  h1 += h2;
  h2 += h1;
  h1 = fmix(h1);
  h2 = fmix(h2);
  h1 += h2;
  return (int32_t)(uint32_t)(h1 & 0xffffffffULL);
}

inline int guavaConsistentHash(int64_t input, int buckets) {
  int64_t state = input;
  int candidate = 0;
  while (true) {
    state = (int64_t)(2862933555777941757ULL * (uint64_t)state + 1ULL);
    const double nextDouble = (double)((int32_t)((uint64_t)state >> 33) + 1) / 2147483648.0;
    const double d = (double)(candidate + 1) / nextDouble;
    int next;
    if (d != d) next = 0;  // Java (int) narrowing: NaN -> 0, saturating at the int range
    else if (d >= 2147483647.0) next = 2147483647;
    else next = (int)d;
    if (next >= 0 && next < buckets) candidate = next;
    else return candidate;
  }
}

inline int topicNameHashBucket(const std::string& topic, int numSets) {
  const int32_t h = guavaMurmur3AsInt(topic);
  const int32_t a = h == INT32_MIN ? h : (h < 0 ? -h : h);  // Math.abs(int)
  return guavaConsistentHash((int64_t)a, numSets);
}

}  // namespace oracle
