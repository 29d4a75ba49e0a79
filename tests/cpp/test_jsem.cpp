// Unit checks of the Java-collection emulations in engine/jsem.h that the drivers rely on (built and run by
// tests/test_jsem_cpp.py, CPU only):
//  * RbTreeSet::buildByRank (puts placed by rank, no comparator walk) builds the same structure as the same put
//    sequence through add() with a comparator, with and without its in-order sequence;
//  * the in-order sequence an RbTreeSet maintains through add / remove equals a walk of the tree;
//  * OrderedQueue: polling up to an element in runs (runBefore(heapPeek) + skipRun + heapPoll, the leadership move-in's
//    bulk polls) visits the elements in the order poll() does.
#include <cstdio>
#include <random>
#include <vector>

#include "jsem.h"

using namespace ccmi;

static int fails = 0;
#define CHECK(c, ...)                        \
  do {                                       \
    if (!(c)) {                              \
      std::fprintf(stderr, __VA_ARGS__);     \
      std::fprintf(stderr, "\n");            \
      ++fails;                               \
    }                                        \
  } while (0)

struct RankCmp {
  const std::vector<int32_t>* rank;
  int operator()(int a, int b) const { return (*rank)[a] < (*rank)[b] ? -1 : ((*rank)[a] > (*rank)[b] ? 1 : 0); }
};
struct NoCmp {
  int operator()(int, int) const { return 0; }
};

static void buildByRankMatchesAdd(std::mt19937& g, int B, int n) {
  std::vector<int> perm(B);
  for (int i = 0; i < B; ++i) perm[i] = i;
  std::shuffle(perm.begin(), perm.end(), g);
  std::vector<int32_t> rank(B, 0);
  std::vector<uint8_t> in(B, 0);
  for (int i = 0; i < n; ++i) {
    rank[perm[i]] = i;
    in[perm[i]] = 1;
  }
  std::vector<int> ids;
  for (int x = 0; x < B; ++x)
    if (in[x]) ids.push_back(x);
  RbTreeSet<RankCmp> byAdd(RankCmp{&rank});
  for (int x : ids) byAdd.add(x);
  for (int withSeq = 0; withSeq < 2; ++withSeq) {
    RbTreeSet<NoCmp> built(NoCmp{});
    std::vector<int> i2(ids);
    std::vector<int32_t> r2(rank);
    built.buildByRank(std::move(i2), std::move(r2), nullptr, withSeq != 0);
    CHECK(built.shapeHash() == byAdd.shapeHash(), "buildByRank shape differs (B=%d n=%d seq=%d)", B, n, withSeq);
    CHECK((built.sequence() != nullptr) == (withSeq != 0), "buildByRank sequence flag (seq=%d)", withSeq);
    if (withSeq) {
      std::vector<int> walk;
      byAdd.inorder(walk);
      CHECK(*built.sequence() == walk, "buildByRank sequence differs from the in-order walk (n=%d)", n);
    }
  }
}

static void sequenceThroughChanges(std::mt19937& g, int B) {
  std::vector<int32_t> rank(B);
  for (int i = 0; i < B; ++i) rank[i] = i;
  std::shuffle(rank.begin(), rank.end(), g);
  RbTreeSet<RankCmp> t(RankCmp{&rank});
  for (int x = 0; x < B; x += 2) t.add(x);
  t.trackSequence();
  std::uniform_int_distribution<int> pick(0, B - 1);
  for (int step = 0; step < 400; ++step) {
    const int x = pick(g);
    if (step % 3 == 0) t.remove(x);
    else t.add(x);
    const std::vector<int> seq = *t.sequence();
    t.untrackSequence();
    std::vector<int> walk;
    t.inorder(walk);
    t.trackSequence();
    CHECK(seq == walk, "maintained sequence differs from the walk at step %d", step);
    if (seq != walk) return;
  }
}

static void bulkPollsMatchPolls(std::mt19937& g, int n) {
  std::vector<int> key(n);
  for (int i = 0; i < n; ++i) key[i] = i;
  std::shuffle(key.begin(), key.end(), g);
  auto cmp = [&key](int a, int b) { return key[a] < key[b] ? -1 : (key[a] > key[b] ? 1 : 0); };
  OrderedQueue<decltype(cmp)> a(cmp), b(cmp);
  std::vector<int> run;
  for (int x = 0; x < n; ++x)
    if (x % 4 != 0) run.push_back(x);
  std::sort(run.begin(), run.end(), [&](int x, int y) { return cmp(x, y) < 0; });
  a.sorted() = run;
  b.sorted() = run;
  for (int x = 0; x < n; x += 8) {  // re-added elements in the heap
    a.add(x);
    b.add(x);
  }
  std::uniform_int_distribution<int> gap(0, 12);
  while (!a.empty()) {
    // the target: some element ahead in poll order (poll a copy of the queue to find it)
    OrderedQueue<decltype(cmp)> c = a;
    int target = -1;
    for (int k = gap(g); k >= 0 && !c.empty(); --k) target = c.poll();
    // naive polls up to the target
    std::vector<int> naive, bulk;
    for (;;) {
      const int x = a.poll();
      naive.push_back(x);
      if (x == target) break;
    }
    // bulk polls: the run's elements before the heap's next one in one pass, then that one
    for (bool found = false; !found;) {
      const bool heapEmpty = b.heapEmpty();
      const size_t k = heapEmpty ? b.runLeft() : b.runBefore(b.heapPeek());
      const int* r = b.runData();
      size_t j = 0;
      while (j < k && r[j] != target) ++j;
      for (size_t q = 0; q < std::min(j + 1, k); ++q) bulk.push_back(r[q]);
      if (j < k) {
        b.skipRun(j + 1);
        found = true;
        break;
      }
      b.skipRun(k);
      if (heapEmpty) break;
      const int h = b.heapPoll();
      bulk.push_back(h);
      found = h == target;
    }
    CHECK(naive == bulk, "bulk polls differ from polls (n=%d, target %d)", n, target);
    if (naive != bulk) return;
    if (!a.empty() && gap(g) < 3) {  // re-add the polled target with a new key behind the head
      key[target] = key[a.peek()] + n + gap(g);
      a.add(target);
      b.add(target);
    }
  }
  CHECK(b.empty(), "bulk-polled queue not empty (n=%d)", n);
}

int main() {
  std::mt19937 g(12345);
  for (int n : {1, 2, 3, 17, 100, 999, 3000}) buildByRankMatchesAdd(g, n + 37, n);
  for (int B : {10, 200, 2000}) sequenceThroughChanges(g, B);
  for (int n : {5, 64, 500, 4000}) bulkPollsMatchPolls(g, n);
  if (fails) {
    std::fprintf(stderr, "%d check(s) failed\n", fails);
    return 1;
  }
  std::printf("jsem ok\n");
  return 0;
}
