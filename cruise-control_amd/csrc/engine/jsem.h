// Java-semantics core for the engine's host driver (product code).
//
// The goal drivers must reproduce the reference's decisions bit for bit, and several JDK 11 collection
// and math behaviours leak into those decisions:
//   * Math.max / Double.compare sign-of-zero and NaN rules;
//   * java.util.TreeMap red-black tree whose comparator reads LIVE broker state, so a node whose key
//     changed is found (or missed) along the comparator path exactly as the JDK would
//     (ResourceDistributionGoal.java:787-793,852-855; ReplicaDistributionGoal.java:232-268);
//   * java.util.PriorityQueue sift order (ResourceDistributionGoal.java:452,630,720);
//   * iteration order of HashSet<Broker> built by Collectors.toSet() (Broker.hashCode() == id);
//   * java.util.Random (fixture generator, RandomCluster.java:465-478).
// The tree is kept in flat struct-of-arrays form (parent/left/right/key/colour vectors) so an in-order
// snapshot for a device scan is one linear walk.
#pragma once
#include <cstdint>
#include <cstring>
#include <cmath>
#include <stdexcept>
#include <vector>

namespace ccmi {

inline double jmax(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && std::signbit(a)) return b;
  return a >= b ? a : b;
}
inline double jmin(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && std::signbit(b)) return b;
  return a <= b ? a : b;
}
inline int jcmpDouble(double a, double b) {  // Double.compare
  if (a < b) return -1;
  if (a > b) return 1;
  int64_t x, y;
  if (a != a) x = 0x7ff8000000000000LL; else std::memcpy(&x, &a, 8);
  if (b != b) y = 0x7ff8000000000000LL; else std::memcpy(&y, &b, 8);
  return x == y ? 0 : (x < y ? -1 : 1);
}
inline int jcmpInt(int64_t a, int64_t b) { return a < b ? -1 : (a > b ? 1 : 0); }

struct JavaRandom {
  uint64_t seed;
  explicit JavaRandom(int64_t s) : seed(((uint64_t)s ^ 0x5DEECE66DULL) & ((1ULL << 48) - 1)) {}
  int32_t next(int bits) {
    seed = (seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1);
    return (int32_t)(seed >> (48 - bits));
  }
  int32_t nextInt(int32_t bound) {
    int32_t r = next(31);
    int32_t m = bound - 1;
    if ((bound & m) == 0) return (int32_t)(((int64_t)bound * (int64_t)r) >> 31);
    uint32_t u = (uint32_t)r;
    for (;;) {
      r = (int32_t)(u % (uint32_t)bound);
      if ((int32_t)(u - (uint32_t)r + (uint32_t)m) >= 0) break;
      u = (uint32_t)next(31);
    }
    return r;
  }
  double nextDouble() {
    int64_t hi = next(26);
    int64_t lo = next(27);
    return (double)((hi << 27) + lo) * (1.0 / 9007199254740992.0);
  }
};

// ----------------------------------------------------------------------------------------------
// java.util.TreeMap<Integer-like key> with an external live comparator. Cmp: int(int a, int b).
template <class Cmp>
class RbTreeSet {
 public:
  explicit RbTreeSet(Cmp c) : cmp_(c) {}
  int size() const { return size_; }
  bool add(int k) {
    int t = root_;
    if (t < 0) {
      root_ = alloc(k, -1);
      size_ = 1;
      return true;
    }
    int parent = -1, c = 0;
    while (t >= 0) {
      parent = t;
      c = cmp_(k, key_[t]);
      if (c < 0) t = left_[t];
      else if (c > 0) t = right_[t];
      else return false;
    }
    int e = alloc(k, parent);
    (c < 0 ? left_[parent] : right_[parent]) = e;
    insertFix(e);
    ++size_;
    return true;
  }
  // Insert `ids` in order into an EMPTY tree whose comparator agrees with `rank` (distinct ranks) on these
  // elements: the same sequence of TreeMap.put calls and therefore the same structure, with integer compares.
  void buildByRank(const std::vector<int>& ids, const std::vector<int32_t>& rank) {
    const size_t n = ids.size();
    key_.reserve(n);
    left_.reserve(n);
    right_.reserve(n);
    parent_.reserve(n);
    red_.reserve(n);
    nodeRank_.resize(n);
    for (int k : ids) {
      const int32_t rk = rank[k];
      if (root_ < 0) {
        root_ = alloc(k, -1);
        nodeRank_[root_] = rk;
        size_ = 1;
        continue;
      }
      int t = root_, parent = -1;
      bool goLeft = false;
      while (t >= 0) {
        parent = t;
        goLeft = rk < nodeRank_[t];
        t = goLeft ? left_[t] : right_[t];
      }
      const int e = alloc(k, parent);
      nodeRank_[e] = rk;
      (goLeft ? left_[parent] : right_[parent]) = e;
      insertFix(e);
      ++size_;
    }
  }
  bool remove(int k) {
    int p = find(k);
    if (p < 0) return false;
    erase(p);
    return true;
  }
  bool contains(int k) const { return find(k) >= 0; }
  void inorder(std::vector<int>& out) const {
    out.clear();
    int p = root_;
    if (p < 0) return;
    while (left_[p] >= 0) p = left_[p];
    for (; p >= 0; p = succ(p)) out.push_back(key_[p]);
  }

 private:
  Cmp cmp_;
  std::vector<int> key_, left_, right_, parent_;
  std::vector<int32_t> nodeRank_;  // buildByRank only
  std::vector<uint8_t> red_;
  std::vector<int> free_;
  int root_ = -1, size_ = 0;

  int alloc(int k, int parent) {
    int id;
    if (!free_.empty()) {
      id = free_.back();
      free_.pop_back();
      key_[id] = k;
      left_[id] = right_[id] = -1;
      parent_[id] = parent;
      red_[id] = 0;
    } else {
      id = (int)key_.size();
      key_.push_back(k);
      left_.push_back(-1);
      right_.push_back(-1);
      parent_.push_back(parent);
      red_.push_back(0);
    }
    return id;
  }
  int find(int k) const {
    int p = root_;
    while (p >= 0) {
      int c = cmp_(k, key_[p]);
      if (c == 0) return p;
      p = c < 0 ? left_[p] : right_[p];
    }
    return -1;
  }
  int succ(int t) const {
    if (right_[t] >= 0) {
      int p = right_[t];
      while (left_[p] >= 0) p = left_[p];
      return p;
    }
    int p = parent_[t], ch = t;
    while (p >= 0 && ch == right_[p]) {
      ch = p;
      p = parent_[p];
    }
    return p;
  }
  bool isRed(int p) const { return p >= 0 && red_[p]; }
  int par(int p) const { return p < 0 ? -1 : parent_[p]; }
  int lft(int p) const { return p < 0 ? -1 : left_[p]; }
  int rgt(int p) const { return p < 0 ? -1 : right_[p]; }
  void paint(int p, bool red) {
    if (p >= 0) red_[p] = red;
  }
  void rotL(int p) {
    if (p < 0) return;
    int r = right_[p];
    right_[p] = left_[r];
    if (left_[r] >= 0) parent_[left_[r]] = p;
    parent_[r] = parent_[p];
    if (parent_[p] < 0) root_ = r;
    else if (left_[parent_[p]] == p) left_[parent_[p]] = r;
    else right_[parent_[p]] = r;
    left_[r] = p;
    parent_[p] = r;
  }
  void rotR(int p) {
    if (p < 0) return;
    int l = left_[p];
    left_[p] = right_[l];
    if (right_[l] >= 0) parent_[right_[l]] = p;
    parent_[l] = parent_[p];
    if (parent_[p] < 0) root_ = l;
    else if (right_[parent_[p]] == p) right_[parent_[p]] = l;
    else left_[parent_[p]] = l;
    right_[l] = p;
    parent_[p] = l;
  }
  // TreeMap.fixAfterInsertion
  void insertFix(int x) {
    red_[x] = 1;
    while (x >= 0 && x != root_ && red_[parent_[x]]) {
      int g = par(par(x));
      if (par(x) == lft(g)) {
        int y = rgt(g);
        if (isRed(y)) {
          paint(par(x), false);
          paint(y, false);
          paint(g, true);
          x = g;
        } else {
          if (x == rgt(par(x))) {
            x = par(x);
            rotL(x);
          }
          paint(par(x), false);
          paint(par(par(x)), true);
          rotR(par(par(x)));
        }
      } else {
        int y = lft(g);
        if (isRed(y)) {
          paint(par(x), false);
          paint(y, false);
          paint(g, true);
          x = g;
        } else {
          if (x == lft(par(x))) {
            x = par(x);
            rotR(x);
          }
          paint(par(x), false);
          paint(par(par(x)), true);
          rotL(par(par(x)));
        }
      }
    }
    red_[root_] = 0;
  }
  // TreeMap.deleteEntry (successor key copied into the doomed node) + fixAfterDeletion
  void erase(int p) {
    --size_;
    if (left_[p] >= 0 && right_[p] >= 0) {
      int s = succ(p);
      key_[p] = key_[s];
      p = s;
    }
    int rep = left_[p] >= 0 ? left_[p] : right_[p];
    if (rep >= 0) {
      parent_[rep] = parent_[p];
      if (parent_[p] < 0) root_ = rep;
      else if (p == left_[parent_[p]]) left_[parent_[p]] = rep;
      else right_[parent_[p]] = rep;
      left_[p] = right_[p] = parent_[p] = -1;
      if (!red_[p]) deleteFix(rep);
    } else if (parent_[p] < 0) {
      root_ = -1;
    } else {
      if (!red_[p]) deleteFix(p);
      int pp = parent_[p];
      if (pp >= 0) {
        if (p == left_[pp]) left_[pp] = -1;
        else if (p == right_[pp]) right_[pp] = -1;
        parent_[p] = -1;
      }
    }
    free_.push_back(p);
  }
  void deleteFix(int x) {
    while (x != root_ && !isRed(x)) {
      if (x == lft(par(x))) {
        int sib = rgt(par(x));
        if (isRed(sib)) {
          paint(sib, false);
          paint(par(x), true);
          rotL(par(x));
          sib = rgt(par(x));
        }
        if (!isRed(lft(sib)) && !isRed(rgt(sib))) {
          paint(sib, true);
          x = par(x);
        } else {
          if (!isRed(rgt(sib))) {
            paint(lft(sib), false);
            paint(sib, true);
            rotR(sib);
            sib = rgt(par(x));
          }
          paint(sib, isRed(par(x)));
          paint(par(x), false);
          paint(rgt(sib), false);
          rotL(par(x));
          x = root_;
        }
      } else {
        int sib = lft(par(x));
        if (isRed(sib)) {
          paint(sib, false);
          paint(par(x), true);
          rotR(par(x));
          sib = lft(par(x));
        }
        if (!isRed(rgt(sib)) && !isRed(lft(sib))) {
          paint(sib, true);
          x = par(x);
        } else {
          if (!isRed(lft(sib))) {
            paint(rgt(sib), false);
            paint(sib, true);
            rotL(sib);
            sib = lft(par(x));
          }
          paint(sib, isRed(par(x)));
          paint(par(x), false);
          paint(lft(sib), false);
          rotR(par(x));
          x = root_;
        }
      }
    }
    paint(x, false);
  }
};

// java.util.PriorityQueue<Integer-like> with comparator.
template <class Cmp>
class JavaPQ {
 public:
  explicit JavaPQ(Cmp c) : cmp_(c) {}
  bool empty() const { return h_.empty(); }
  int size() const { return (int)h_.size(); }
  int peek() const { return h_[0]; }
  void add(int x) {
    int k = (int)h_.size();
    h_.push_back(x);
    while (k > 0) {
      int parent = (k - 1) >> 1;
      if (cmp_(x, h_[parent]) >= 0) break;
      h_[k] = h_[parent];
      k = parent;
    }
    h_[k] = x;
  }
  int poll() {
    int top = h_[0];
    int x = h_.back();
    h_.pop_back();
    int n = (int)h_.size();
    if (n > 0) {
      int k = 0, half = n >> 1;
      while (k < half) {
        int c = 2 * k + 1;
        if (c + 1 < n && cmp_(h_[c], h_[c + 1]) > 0) ++c;
        if (cmp_(x, h_[c]) <= 0) break;
        h_[k] = h_[c];
        k = c;
      }
      h_[k] = x;
    }
    return top;
  }

 private:
  Cmp cmp_;
  std::vector<int> h_;
};

// A java.util.PriorityQueue whose elements never change key while they are queued polls in ascending
// comparator order (the heap invariant always holds and the comparator is a total order). OrderedQueue is that
// queue built in O(n): a cursor over the members presorted by the caller plus a JavaPQ for elements added later.
// Callers must fall back to JavaPQ when a queued element's key can change (stale-key heap semantics).
template <class Cmp>
class OrderedQueue {
 public:
  explicit OrderedQueue(Cmp c) : cmp_(c), heap_(c) {}
  std::vector<int>& sorted() { return s_; }  // members in ascending comparator order, filled before use
  bool empty() const { return pos_ >= s_.size() && heap_.empty(); }
  int peek() const {
    if (heap_.empty()) return s_[pos_];
    if (pos_ >= s_.size()) return heap_.peek();
    return cmp_(heap_.peek(), s_[pos_]) < 0 ? heap_.peek() : s_[pos_];
  }
  int poll() {
    if (heap_.empty()) return s_[pos_++];
    if (pos_ >= s_.size()) return heap_.poll();
    if (cmp_(heap_.peek(), s_[pos_]) < 0) return heap_.poll();
    return s_[pos_++];
  }
  void add(int x) { heap_.add(x); }

 private:
  Cmp cmp_;
  JavaPQ<Cmp> heap_;
  std::vector<int> s_;
  size_t pos_ = 0;
};

// Iteration order of a HashSet<Broker> filled by add() in `ins` order (Broker.hashCode() == id).
inline void javaHashSetOrder(const std::vector<int>& ins, std::vector<int>& out) {
  unsigned cap = 16;
  size_t n = 0;
  std::vector<std::vector<int>> bins(cap);
  auto slot = [](int h, unsigned c) { return (unsigned)(h ^ (int)((unsigned)h >> 16)) & (c - 1); };
  auto grow = [&]() {
    unsigned nc = cap << 1;
    std::vector<std::vector<int>> nb(nc);
    for (auto& b : bins)
      for (int k : b) nb[slot(k, nc)].push_back(k);
    bins.swap(nb);
    cap = nc;
  };
  for (int k : ins) {
    auto& b = bins[slot(k, cap)];
    bool dup = false;
    for (int x : b) dup |= (x == k);
    if (dup) continue;
    b.push_back(k);
    if (b.size() >= 9) {
      if (cap < 64) grow();
      else throw std::runtime_error("HashSet tree bin order is not emulated");
    }
    if (++n > (size_t)(cap * 3 / 4)) grow();
  }
  out.clear();
  for (auto& b : bins)
    for (int k : b) out.push_back(k);
}

}  // namespace ccmi
