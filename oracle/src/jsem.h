// ORACLE — test infrastructure only. Never linked into, imported by, or executed from the
// product path (cruise-control_amd/). Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may use it, and only as the checker / CPU baseline.
//
// jsem.h — the handful of JDK 11 semantics that leak into Cruise Control's optimizer results.
//   * java.util.Random (JDK 11 java/util/Random.java: setSeed/next/nextInt(bound)/nextDouble)
//     used by RandomCluster.uniformlyRandom / exponentialRandom
//     (cruise-control/src/test/.../model/RandomCluster.java:465-478).
//   * Math.max/Math.min/Double.compare sign-of-zero and NaN rules.
//   * java.util.TreeMap red-black tree (CLR insert/delete with successor-copy, comparator-path
//     lookup with LIVE keys), needed because candidate-broker TreeSets are keyed on mutable
//     utilization and patched with remove/add after every accepted move
//     (ResourceDistributionGoal.java:787-793,852-855; ReplicaDistributionGoal.java:232-238,266-268).
//   * java.util.PriorityQueue binary heap (siftUp/siftDown using comparator)
//     (ResourceDistributionGoal.java:452,630,720; ReplicaDistributionGoal.java:283-291).
//   * DoubleStream.sum() compensated summation, JDK 11 flavour (Collectors.sumWithCompensation +
//     computeFinalSum = sum + compensation), used by ClusterModelStats.java utilizationForPotentialNwOut.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>
#include <functional>
#include <stdexcept>

namespace oracle {

// ---------------------------------------------------------------- java.util.Random
struct JRandom {
  int64_t seed;
  explicit JRandom(int64_t s) { seed = (s ^ 0x5DEECE66DLL) & ((1LL << 48) - 1); }
  int32_t next(int bits) {
    seed = (int64_t)(((uint64_t)seed * 0x5DEECE66DULL + 0xBULL) & ((1ULL << 48) - 1));
    return (int32_t)((uint64_t)seed >> (48 - bits));
  }
  int32_t nextInt(int32_t bound) {
    if (bound <= 0) throw std::invalid_argument("bound must be positive");
    int32_t r = next(31);
    int32_t m = bound - 1;
    if ((bound & m) == 0) {
      r = (int32_t)(((int64_t)bound * (int64_t)r) >> 31);
    } else {
      for (int32_t u = r; (int32_t)((uint32_t)u - (uint32_t)(r = u % bound) + (uint32_t)m) < 0; u = next(31)) {
      }
    }
    return r;
  }
  double nextDouble() {
    int64_t hi = (int64_t)next(26);
    int64_t lo = (int64_t)next(27);
    return (double)((hi << 27) + lo) * 0x1.0p-53;
  }
};

// ---------------------------------------------------------------- Math / Double semantics
inline bool isNegZero(double d) { return d == 0.0 && std::signbit(d); }
inline double jmax(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && isNegZero(a)) return b;
  return (a >= b) ? a : b;
}
inline double jmin(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && isNegZero(b)) return b;
  return (a <= b) ? a : b;
}
inline float jmaxf(float a, float b) {
  if (a != a) return a;
  if (a == 0.0f && b == 0.0f && std::signbit(a)) return b;
  return (a >= b) ? a : b;
}
// Double.compare: -0.0 < 0.0, NaN == NaN and greater than everything.
inline int64_t jDoubleToLongBits(double d) {
  if (d != d) return 0x7ff8000000000000LL;
  int64_t b;
  std::memcpy(&b, &d, 8);
  return b;
}
inline int dcompare(double a, double b) {
  if (a < b) return -1;
  if (a > b) return 1;
  int64_t x = jDoubleToLongBits(a), y = jDoubleToLongBits(b);
  return x == y ? 0 : (x < y ? -1 : 1);
}
inline int icompare(int64_t a, int64_t b) { return a < b ? -1 : (a > b ? 1 : 0); }

// DoubleStream.sum() in JDK 11 (compensated; final = sum + compensation).
struct JDoubleSum {
  double s0 = 0.0, s1 = 0.0, simple = 0.0;
  void add(double v) {
    double tmp = v - s1;
    double sum = s0;
    double velvel = sum + tmp;
    s1 = (velvel - sum) - tmp;
    s0 = velvel;
    simple += v;
  }
  double result() const {
    double tmp = s0 + s1;
    if (std::isnan(tmp) && std::isinf(simple)) return simple;
    return tmp;
  }
};

// ---------------------------------------------------------------- java.util.TreeMap (as TreeSet<int>)
// Keys are small ints (broker ids / replica indices). The comparator reads LIVE state, so stale
// nodes behave exactly as in the JDK: lookups follow the comparator path and may miss them.
class JTreeSet {
 public:
  using Cmp = std::function<int(int, int)>;
  explicit JTreeSet(Cmp cmp) : cmp_(std::move(cmp)) {}

  int size() const { return size_; }
  bool empty() const { return size_ == 0; }

  // TreeSet.add -> TreeMap.put; returns true if inserted.
  bool add(int key) {
    int t = root_;
    if (t < 0) {
      cmp_(key, key);
      root_ = newNode(key, -1);
      size_ = 1;
      return true;
    }
    int c = 0, parent;
    do {
      parent = t;
      c = cmp_(key, nodes_[t].key);
      if (c < 0) t = nodes_[t].left;
      else if (c > 0) t = nodes_[t].right;
      else return false;
    } while (t >= 0);
    int e = newNode(key, parent);
    if (c < 0) nodes_[parent].left = e;
    else nodes_[parent].right = e;
    fixAfterInsertion(e);
    size_++;
    return true;
  }
  // TreeSet.remove -> TreeMap.remove (getEntryUsingComparator + deleteEntry).
  bool remove(int key) {
    int p = getEntry(key);
    if (p < 0) return false;
    deleteEntry(p);
    return true;
  }
  bool contains(int key) const { return getEntry(key) >= 0; }
  // Collection.removeIf over the TreeSet iterator (no comparator: stale nodes are found too). TreeMap's
  // PrivateEntryIterator.remove continues at the removed entry when it had two children: deleteEntry moved the
  // successor's key into it.
  template <class Pred>
  bool removeIf(Pred pred) {
    bool removed = false;
    for (int e = firstEntry(); e >= 0;) {
      int next = successor(e);
      if (pred(nodes_[e].key)) {
        if (nodes_[e].left >= 0 && nodes_[e].right >= 0) next = e;
        deleteEntry(e);
        removed = true;
      }
      e = next;
    }
    return removed;
  }

  // In-order iteration (TreeMap iterator: getFirstEntry + successor).
  std::vector<int> toVector() const {
    std::vector<int> out;
    toVector(out);
    return out;
  }
  void toVector(std::vector<int>& out) const {
    out.clear();
    out.reserve(size_);
    for (int e = firstEntry(); e >= 0; e = successor(e)) out.push_back(nodes_[e].key);
  }
  int first() const {
    int e = firstEntry();
    if (e < 0) throw std::runtime_error("NoSuchElement");
    return nodes_[e].key;
  }
  // Debug/validation: returns the sequence of (key) in order.

 private:
  struct Node {
    int key, left, right, parent;
    bool black;
  };
  std::vector<Node> nodes_;
  std::vector<int> free_;
  int root_ = -1;
  int size_ = 0;
  Cmp cmp_;

  int newNode(int key, int parent) {
    int id;
    if (!free_.empty()) {
      id = free_.back();
      free_.pop_back();
    } else {
      id = (int)nodes_.size();
      nodes_.push_back({});
    }
    nodes_[id] = {key, -1, -1, parent, true};  // Entry() is BLACK by default
    return id;
  }
  int getEntry(int key) const {
    int p = root_;
    while (p >= 0) {
      int c = cmp_(key, nodes_[p].key);
      if (c < 0) p = nodes_[p].left;
      else if (c > 0) p = nodes_[p].right;
      else return p;
    }
    return -1;
  }
  int firstEntry() const {
    int p = root_;
    if (p >= 0)
      while (nodes_[p].left >= 0) p = nodes_[p].left;
    return p;
  }
  int successor(int t) const {
    if (t < 0) return -1;
    if (nodes_[t].right >= 0) {
      int p = nodes_[t].right;
      while (nodes_[p].left >= 0) p = nodes_[p].left;
      return p;
    }
    int p = nodes_[t].parent, ch = t;
    while (p >= 0 && ch == nodes_[p].right) {
      ch = p;
      p = nodes_[p].parent;
    }
    return p;
  }
  // null-safe helpers as in TreeMap
  bool colorOf(int p) const { return p < 0 ? true : nodes_[p].black; }  // true == BLACK
  int parentOf(int p) const { return p < 0 ? -1 : nodes_[p].parent; }
  void setColor(int p, bool black) {
    if (p >= 0) nodes_[p].black = black;
  }
  int leftOf(int p) const { return p < 0 ? -1 : nodes_[p].left; }
  int rightOf(int p) const { return p < 0 ? -1 : nodes_[p].right; }
  void rotateLeft(int p) {
    if (p < 0) return;
    int r = nodes_[p].right;
    nodes_[p].right = nodes_[r].left;
    if (nodes_[r].left >= 0) nodes_[nodes_[r].left].parent = p;
    nodes_[r].parent = nodes_[p].parent;
    if (nodes_[p].parent < 0) root_ = r;
    else if (nodes_[nodes_[p].parent].left == p) nodes_[nodes_[p].parent].left = r;
    else nodes_[nodes_[p].parent].right = r;
    nodes_[r].left = p;
    nodes_[p].parent = r;
  }
  void rotateRight(int p) {
    if (p < 0) return;
    int l = nodes_[p].left;
    nodes_[p].left = nodes_[l].right;
    if (nodes_[l].right >= 0) nodes_[nodes_[l].right].parent = p;
    nodes_[l].parent = nodes_[p].parent;
    if (nodes_[p].parent < 0) root_ = l;
    else if (nodes_[nodes_[p].parent].right == p) nodes_[nodes_[p].parent].right = l;
    else nodes_[nodes_[p].parent].left = l;
    nodes_[l].right = p;
    nodes_[p].parent = l;
  }
  void fixAfterInsertion(int x) {
    nodes_[x].black = false;
    while (x >= 0 && x != root_ && !nodes_[nodes_[x].parent].black) {
      if (parentOf(x) == leftOf(parentOf(parentOf(x)))) {
        int y = rightOf(parentOf(parentOf(x)));
        if (!colorOf(y)) {
          setColor(parentOf(x), true);
          setColor(y, true);
          setColor(parentOf(parentOf(x)), false);
          x = parentOf(parentOf(x));
        } else {
          if (x == rightOf(parentOf(x))) {
            x = parentOf(x);
            rotateLeft(x);
          }
          setColor(parentOf(x), true);
          setColor(parentOf(parentOf(x)), false);
          rotateRight(parentOf(parentOf(x)));
        }
      } else {
        int y = leftOf(parentOf(parentOf(x)));
        if (!colorOf(y)) {
          setColor(parentOf(x), true);
          setColor(y, true);
          setColor(parentOf(parentOf(x)), false);
          x = parentOf(parentOf(x));
        } else {
          if (x == leftOf(parentOf(x))) {
            x = parentOf(x);
            rotateRight(x);
          }
          setColor(parentOf(x), true);
          setColor(parentOf(parentOf(x)), false);
          rotateLeft(parentOf(parentOf(x)));
        }
      }
    }
    nodes_[root_].black = true;
  }
  void deleteEntry(int p) {
    size_--;
    if (nodes_[p].left >= 0 && nodes_[p].right >= 0) {
      int s = successor(p);
      nodes_[p].key = nodes_[s].key;
      p = s;
    }
    int replacement = nodes_[p].left >= 0 ? nodes_[p].left : nodes_[p].right;
    if (replacement >= 0) {
      nodes_[replacement].parent = nodes_[p].parent;
      if (nodes_[p].parent < 0) root_ = replacement;
      else if (p == nodes_[nodes_[p].parent].left) nodes_[nodes_[p].parent].left = replacement;
      else nodes_[nodes_[p].parent].right = replacement;
      nodes_[p].left = nodes_[p].right = nodes_[p].parent = -1;
      if (nodes_[p].black) fixAfterDeletion(replacement);
    } else if (nodes_[p].parent < 0) {
      root_ = -1;
    } else {
      if (nodes_[p].black) fixAfterDeletion(p);
      if (nodes_[p].parent >= 0) {
        int pp = nodes_[p].parent;
        if (p == nodes_[pp].left) nodes_[pp].left = -1;
        else if (p == nodes_[pp].right) nodes_[pp].right = -1;
        nodes_[p].parent = -1;
      }
    }
    free_.push_back(p);
  }
  void fixAfterDeletion(int x) {
    while (x != root_ && colorOf(x)) {
      if (x == leftOf(parentOf(x))) {
        int sib = rightOf(parentOf(x));
        if (!colorOf(sib)) {
          setColor(sib, true);
          setColor(parentOf(x), false);
          rotateLeft(parentOf(x));
          sib = rightOf(parentOf(x));
        }
        if (colorOf(leftOf(sib)) && colorOf(rightOf(sib))) {
          setColor(sib, false);
          x = parentOf(x);
        } else {
          if (colorOf(rightOf(sib))) {
            setColor(leftOf(sib), true);
            setColor(sib, false);
            rotateRight(sib);
            sib = rightOf(parentOf(x));
          }
          setColor(sib, colorOf(parentOf(x)));
          setColor(parentOf(x), true);
          setColor(rightOf(sib), true);
          rotateLeft(parentOf(x));
          x = root_;
        }
      } else {
        int sib = leftOf(parentOf(x));
        if (!colorOf(sib)) {
          setColor(sib, true);
          setColor(parentOf(x), false);
          rotateRight(parentOf(x));
          sib = leftOf(parentOf(x));
        }
        if (colorOf(rightOf(sib)) && colorOf(leftOf(sib))) {
          setColor(sib, false);
          x = parentOf(x);
        } else {
          if (colorOf(leftOf(sib))) {
            setColor(rightOf(sib), true);
            setColor(sib, false);
            rotateLeft(sib);
            sib = leftOf(parentOf(x));
          }
          setColor(sib, colorOf(parentOf(x)));
          setColor(parentOf(x), true);
          setColor(leftOf(sib), true);
          rotateRight(parentOf(x));
          x = root_;
        }
      }
    }
    setColor(x, true);
  }
};

// ---------------------------------------------------------------- java.util.PriorityQueue<int>
class JPriorityQueue {
 public:
  using Cmp = std::function<int(int, int)>;
  explicit JPriorityQueue(Cmp cmp) : cmp_(std::move(cmp)) {}
  bool empty() const { return q_.empty(); }
  int size() const { return (int)q_.size(); }
  void add(int x) {
    int k = (int)q_.size();
    q_.push_back(x);
    while (k > 0) {
      int parent = (k - 1) >> 1;
      int e = q_[parent];
      if (cmp_(x, e) >= 0) break;
      q_[k] = e;
      k = parent;
    }
    q_[k] = x;
  }
  int peek() const { return q_.front(); }
  const std::vector<int>& heap() const { return q_; }
  int poll() {
    int result = q_[0];
    int n = (int)q_.size() - 1;
    int x = q_[n];
    q_.pop_back();
    if (n > 0) {
      int k = 0, half = n >> 1;
      while (k < half) {
        int child = (k << 1) + 1;
        int c = q_[child];
        int right = child + 1;
        if (right < n && cmp_(c, q_[right]) > 0) c = q_[child = right];
        if (cmp_(x, c) <= 0) break;
        q_[k] = c;
        k = child;
      }
      q_[k] = x;
    }
    return result;
  }

 private:
  std::vector<int> q_;
  Cmp cmp_;
};

// ---------------------------------------------------------------- String.hashCode / HashMap
// String.hashCode (JDK: s[0]*31^(n-1) + ... + s[n-1], int arithmetic).
inline int32_t jStringHash(const std::string& s) {
  uint32_t h = 0;
  for (unsigned char c : s) h = 31u * h + (uint32_t)c;
  return (int32_t)h;
}
// Objects.hash-style combination: 31 * h + x with int overflow.
inline int32_t jHashMix(int32_t h, int32_t x) { return (int32_t)(31u * (uint32_t)h + (uint32_t)x); }

// java.util.HashSet<E> (the HashMap<E, PRESENT> behind it, JDK 11 java/util/HashMap.java) for elements
// identified by an int id with a caller-supplied E.hashCode(): power-of-two table allocated lazily,
// hash() spreading, list bins in insertion order, resize splits keeping relative order, TREEIFY at 8+1
// nodes (resize instead below 64 buckets), TreeNode bins with the JDK's red-black tree, next-chain
// insertion after the tree parent, moveRootToFront, removeTreeNode/untreeify and TreeNode.split.
// Equal-hash keys are ordered by `cmp` (compareComparables: E implements Comparable<E>); tieBreakOrder is
// never reached because distinct elements never compare equal.
class JHashSet {
 public:
  using Cmp = std::function<int(int, int)>;
  JHashSet() = default;
  // HashMap(int initialCapacity): threshold = tableSizeFor(initialCapacity), table allocated on first put.
  explicit JHashSet(int initialCapacity, Cmp cmp = nullptr)
      : cmp_(std::move(cmp)), threshold_(tableSizeFor(initialCapacity)) {}
  explicit JHashSet(Cmp cmp) : cmp_(std::move(cmp)) {}
  void setComparator(Cmp cmp) { cmp_ = std::move(cmp); }
  // HashSet(Collection c): new HashMap<>(Math.max((int) (c.size()/.75f) + 1, 16)) then addAll(c)
  static JHashSet copyOf(const JHashSet& src) {
    JHashSet s(std::max((int)((float)src.size() / 0.75f) + 1, 16), src.cmp_);
    for (const auto& e : src.entries()) s.add(e.first, e.second);
    return s;
  }
  static JHashSet copyOf(const std::vector<std::pair<int, int32_t>>& elems, Cmp cmp = nullptr) {
    JHashSet s(std::max((int)((float)elems.size() / 0.75f) + 1, 16), std::move(cmp));
    for (const auto& e : elems) s.add(e.first, e.second);
    return s;
  }
  static int tableSizeFor(int cap) {
    int n = 1;
    while (n < cap) n <<= 1;
    return n;
  }
  static int32_t spread(int32_t h) { return h ^ (int32_t)((uint32_t)h >> 16); }
  int size() const { return size_; }

  bool add(int id, int32_t hashCode) {
    const int32_t h = spread(hashCode);
    if (tab_.empty()) resize();
    int n = (int)tab_.size();
    int i = (n - 1) & h;
    int p = tab_[i];
    if (p < 0) {
      tab_[i] = newNode(id, h, -1);
    } else if (N(p).tree) {
      if (putTreeVal(i, id, h) >= 0) return false;
    } else {
      for (int binCount = 0;; ++binCount) {
        if (N(p).hash == h && N(p).id == id) return false;
        const int e = N(p).next;
        if (e < 0) {
          N(p).next = newNode(id, h, -1);
          if (binCount >= 7) treeifyBin(h);
          break;
        }
        p = e;
      }
    }
    if (++size_ > threshold_) resize();
    return true;
  }
  bool remove(int id, int32_t hashCode) {
    if (tab_.empty()) return false;
    const int32_t h = spread(hashCode);
    const int n = (int)tab_.size(), i = (n - 1) & h;
    int p = tab_[i];
    if (p < 0) return false;
    int node = -1, prevList = -1;
    if (N(p).tree) {
      node = findTree(root(p), h, id);
      if (node < 0) return false;
      removeTreeNode(node);
    } else {
      for (int e = p; e >= 0; prevList = e, e = N(e).next)
        if (N(e).hash == h && N(e).id == id) {
          node = e;
          break;
        }
      if (node < 0) return false;
      if (prevList < 0) tab_[i] = N(node).next;
      else N(prevList).next = N(node).next;
    }
    freeNode(node);
    --size_;
    return true;
  }
  bool contains(int id, int32_t hashCode) const {
    if (tab_.empty()) return false;
    const int32_t h = spread(hashCode);
    int p = tab_[((int)tab_.size() - 1) & h];
    for (; p >= 0; p = nodes_[p].next)
      if (nodes_[p].hash == h && nodes_[p].id == id) return true;
    return false;
  }
  std::vector<int> order() const {
    std::vector<int> out;
    out.reserve(size_);
    for (int head : tab_)
      for (int p = head; p >= 0; p = nodes_[p].next) out.push_back(nodes_[p].id);
    return out;
  }
  // (id, original hashCode is not kept: the spread hash is a bijection's image, so re-spreading it is wrong);
  // entries() returns (id, hashCode) pairs reconstructed by un-spreading.
  std::vector<std::pair<int, int32_t>> entries() const {
    std::vector<std::pair<int, int32_t>> out;
    out.reserve(size_);
    for (int head : tab_)
      for (int p = head; p >= 0; p = nodes_[p].next) out.push_back({nodes_[p].id, unspread(nodes_[p].hash)});
    return out;
  }

 private:
  struct Node {
    int id;
    int32_t hash;
    int next = -1, prev = -1, parent = -1, left = -1, right = -1;
    bool red = false, tree = false;
  };
  std::vector<Node> nodes_;
  std::vector<int> free_;
  std::vector<int> tab_;
  Cmp cmp_;
  int size_ = 0, threshold_ = 0;

  Node& N(int i) { return nodes_[i]; }
  const Node& N(int i) const { return nodes_[i]; }
  // h ^ (h >>> 16) is an involution on the high half, so applying it again restores h
  static int32_t unspread(int32_t s) { return s ^ (int32_t)((uint32_t)s >> 16); }
  int newNode(int id, int32_t h, int next) {
    int k;
    if (!free_.empty()) {
      k = free_.back();
      free_.pop_back();
      nodes_[k] = Node();
    } else {
      k = (int)nodes_.size();
      nodes_.emplace_back();
    }
    nodes_[k].id = id;
    nodes_[k].hash = h;
    nodes_[k].next = next;
    return k;
  }
  void freeNode(int k) { free_.push_back(k); }
  int compareKeys(int a, int b) const { return cmp_ ? cmp_(a, b) : 0; }

  void resize() {
    const int oldCap = (int)tab_.size();
    int newCap;
    if (oldCap > 0) {
      newCap = oldCap << 1;
      threshold_ = (oldCap >= 16) ? threshold_ << 1 : (int)((float)newCap * 0.75f);
    } else if (threshold_ > 0) {
      newCap = threshold_;
      threshold_ = (int)((float)newCap * 0.75f);
    } else {
      newCap = 16;
      threshold_ = 12;
    }
    std::vector<int> old;
    old.swap(tab_);
    tab_.assign(newCap, -1);
    for (int j = 0; j < oldCap; ++j) {
      int e = old[j];
      if (e < 0) continue;
      if (N(e).next < 0) {
        tab_[N(e).hash & (newCap - 1)] = e;
      } else if (N(e).tree) {
        split(e, j, oldCap);
      } else {
        int loH = -1, loT = -1, hiH = -1, hiT = -1;
        for (int next; e >= 0; e = next) {
          next = N(e).next;
          if ((N(e).hash & oldCap) == 0) {
            if (loT < 0) loH = e;
            else N(loT).next = e;
            loT = e;
          } else {
            if (hiT < 0) hiH = e;
            else N(hiT).next = e;
            hiT = e;
          }
        }
        if (loT >= 0) {
          N(loT).next = -1;
          tab_[j] = loH;
        }
        if (hiT >= 0) {
          N(hiT).next = -1;
          tab_[j + oldCap] = hiH;
        }
      }
    }
  }

  void treeifyBin(int32_t h) {
    const int n = (int)tab_.size();
    if (n < 64) {
      resize();
      return;
    }
    const int index = (n - 1) & h;
    int hd = tab_[index], tl = -1;
    for (int e = hd; e >= 0; e = N(e).next) {
      N(e).tree = true;
      N(e).prev = tl;
      tl = e;
    }
    if (hd >= 0) treeify(hd);
  }
  // TreeNode.treeify: insert the chain's nodes in next order, then moveRootToFront
  void treeify(int head) {
    int root = -1;
    for (int x = head, next; x >= 0; x = next) {
      next = N(x).next;
      N(x).left = N(x).right = -1;
      if (root < 0) {
        N(x).parent = -1;
        N(x).red = false;
        root = x;
      } else {
        const int32_t h = N(x).hash;
        for (int p = root;;) {
          int dir;
          const int32_t ph = N(p).hash;
          if (ph > h) dir = -1;
          else if (ph < h) dir = 1;
          else dir = compareKeys(N(x).id, N(p).id) <= 0 ? -1 : 1;
          const int xp = p;
          p = dir <= 0 ? N(p).left : N(p).right;
          if (p < 0) {
            N(x).parent = xp;
            if (dir <= 0) N(xp).left = x;
            else N(xp).right = x;
            root = balanceInsertion(root, x);
            break;
          }
        }
      }
    }
    moveRootToFront(root);
  }
  // untreeify: keep the next-chain order, plain nodes
  void untreeify(int head) {
    for (int e = head; e >= 0; e = N(e).next) {
      N(e).tree = false;
      N(e).parent = N(e).left = N(e).right = N(e).prev = -1;
      N(e).red = false;
    }
  }
  int root(int p) const {
    for (int r = p, q;; r = q)
      if ((q = N(r).parent) < 0) return r;
  }
  void moveRootToFront(int root) {
    if (root < 0 || tab_.empty()) return;
    const int index = ((int)tab_.size() - 1) & N(root).hash;
    const int first = tab_[index];
    if (root != first) {
      tab_[index] = root;
      const int rp = N(root).prev, rn = N(root).next;
      if (rn >= 0) N(rn).prev = rp;
      if (rp >= 0) N(rp).next = rn;
      if (first >= 0) N(first).prev = root;
      N(root).next = first;
      N(root).prev = -1;
    }
  }
  int findTree(int p, int32_t h, int id) const {
    while (p >= 0) {
      const int pl = N(p).left, pr = N(p).right;
      const int32_t ph = N(p).hash;
      if (ph > h) p = pl;
      else if (ph < h) p = pr;
      else if (N(p).id == id) return p;
      else if (pl < 0) p = pr;
      else if (pr < 0) p = pl;
      else {
        const int dir = compareKeys(id, N(p).id);
        if (dir != 0) {
          p = dir < 0 ? pl : pr;
        } else {
          const int q = findTree(pr, h, id);
          if (q >= 0) return q;
          p = pl;
        }
      }
    }
    return -1;
  }
  // TreeNode.putTreeVal: returns the existing node, or -1 after inserting
  int putTreeVal(int index, int id, int32_t h) {
    const int rootNode = root(tab_[index]);
    bool searched = false;
    for (int p = rootNode;;) {
      int dir;
      const int32_t ph = N(p).hash;
      if (ph > h) dir = -1;
      else if (ph < h) dir = 1;
      else if (N(p).id == id) return p;
      else if ((dir = compareKeys(id, N(p).id)) == 0) {
        if (!searched) {
          searched = true;
          int q;
          if ((N(p).left >= 0 && (q = findTree(N(p).left, h, id)) >= 0) ||
              (N(p).right >= 0 && (q = findTree(N(p).right, h, id)) >= 0))
            return q;
        }
        throw std::runtime_error("HashMap tieBreakOrder reached (identityHashCode order is not reproducible)");
      }
      const int xp = p;
      p = dir <= 0 ? N(p).left : N(p).right;
      if (p < 0) {
        const int xpn = N(xp).next;
        const int x = newNode(id, h, xpn);
        N(x).tree = true;
        if (dir <= 0) N(xp).left = x;
        else N(xp).right = x;
        N(xp).next = x;
        N(x).parent = N(x).prev = xp;
        if (xpn >= 0) N(xpn).prev = x;
        moveRootToFront(balanceInsertion(rootNode, x));
        return -1;
      }
    }
  }
  void removeTreeNode(int p) {
    const int n = (int)tab_.size();
    const int index = (n - 1) & N(p).hash;
    int first = tab_[index], rootNode = first;
    const int succ = N(p).next, pred = N(p).prev;
    if (pred < 0) tab_[index] = first = succ;
    else N(pred).next = succ;
    if (succ >= 0) N(succ).prev = pred;
    if (first < 0) return;
    if (N(rootNode).parent >= 0) rootNode = root(rootNode);
    int rl;
    if (rootNode < 0 || N(rootNode).right < 0 || (rl = N(rootNode).left) < 0 || N(rl).left < 0) {
      untreeify(first);  // too small
      return;
    }
    int pl = N(p).left, pr = N(p).right, replacement;
    if (pl >= 0 && pr >= 0) {
      int s = pr, sl;
      while ((sl = N(s).left) >= 0) s = sl;
      const bool c = N(s).red;
      N(s).red = N(p).red;
      N(p).red = c;
      const int sr = N(s).right, pp = N(p).parent;
      if (s == pr) {
        N(p).parent = s;
        N(s).right = p;
      } else {
        const int sp = N(s).parent;
        if ((N(p).parent = sp) >= 0) {
          if (s == N(sp).left) N(sp).left = p;
          else N(sp).right = p;
        }
        if ((N(s).right = pr) >= 0) N(pr).parent = s;
      }
      N(p).left = -1;
      if ((N(p).right = sr) >= 0) N(sr).parent = p;
      if ((N(s).left = pl) >= 0) N(pl).parent = s;
      if ((N(s).parent = pp) < 0) rootNode = s;
      else if (p == N(pp).left) N(pp).left = s;
      else N(pp).right = s;
      replacement = sr >= 0 ? sr : p;
    } else if (pl >= 0) {
      replacement = pl;
    } else if (pr >= 0) {
      replacement = pr;
    } else {
      replacement = p;
    }
    if (replacement != p) {
      const int pp = N(replacement).parent = N(p).parent;
      if (pp < 0) {
        rootNode = replacement;
        N(replacement).red = false;
      } else if (p == N(pp).left) {
        N(pp).left = replacement;
      } else {
        N(pp).right = replacement;
      }
      N(p).left = N(p).right = N(p).parent = -1;
    }
    const int r = N(p).red ? rootNode : balanceDeletion(rootNode, replacement);
    if (replacement == p) {
      const int pp = N(p).parent;
      N(p).parent = -1;
      if (pp >= 0) {
        if (p == N(pp).left) N(pp).left = -1;
        else if (p == N(pp).right) N(pp).right = -1;
      }
    }
    moveRootToFront(r);
  }
  // TreeNode.split during resize
  void split(int b, int index, int bit) {
    int loH = -1, loT = -1, hiH = -1, hiT = -1, lc = 0, hc = 0;
    for (int e = b, next; e >= 0; e = next) {
      next = N(e).next;
      N(e).next = -1;
      if ((N(e).hash & bit) == 0) {
        if ((N(e).prev = loT) < 0) loH = e;
        else N(loT).next = e;
        loT = e;
        ++lc;
      } else {
        if ((N(e).prev = hiT) < 0) hiH = e;
        else N(hiT).next = e;
        hiT = e;
        ++hc;
      }
    }
    if (loH >= 0) {
      if (lc <= 6) {
        untreeify(loH);
        tab_[index] = loH;
      } else {
        tab_[index] = loH;
        if (hiH >= 0) treeify(loH);
      }
    }
    if (hiH >= 0) {
      if (hc <= 6) {
        untreeify(hiH);
        tab_[index + bit] = hiH;
      } else {
        tab_[index + bit] = hiH;
        if (loH >= 0) treeify(hiH);
      }
    }
  }
  int rotateLeft(int root, int p) {
    int r, pp, rl;
    if (p >= 0 && (r = N(p).right) >= 0) {
      if ((rl = N(p).right = N(r).left) >= 0) N(rl).parent = p;
      if ((pp = N(r).parent = N(p).parent) < 0) {
        root = r;
        N(r).red = false;
      } else if (N(pp).left == p) {
        N(pp).left = r;
      } else {
        N(pp).right = r;
      }
      N(r).left = p;
      N(p).parent = r;
    }
    return root;
  }
  int rotateRight(int root, int p) {
    int l, pp, lr;
    if (p >= 0 && (l = N(p).left) >= 0) {
      if ((lr = N(p).left = N(l).right) >= 0) N(lr).parent = p;
      if ((pp = N(l).parent = N(p).parent) < 0) {
        root = l;
        N(l).red = false;
      } else if (N(pp).right == p) {
        N(pp).right = l;
      } else {
        N(pp).left = l;
      }
      N(l).right = p;
      N(p).parent = l;
    }
    return root;
  }
  int balanceInsertion(int root, int x) {
    N(x).red = true;
    for (int xp, xpp, xppl, xppr;;) {
      if ((xp = N(x).parent) < 0) {
        N(x).red = false;
        return x;
      } else if (!N(xp).red || (xpp = N(xp).parent) < 0) {
        return root;
      }
      if (xp == (xppl = N(xpp).left)) {
        if ((xppr = N(xpp).right) >= 0 && N(xppr).red) {
          N(xppr).red = false;
          N(xp).red = false;
          N(xpp).red = true;
          x = xpp;
        } else {
          if (x == N(xp).right) {
            root = rotateLeft(root, x = xp);
            xpp = (xp = N(x).parent) < 0 ? -1 : N(xp).parent;
          }
          if (xp >= 0) {
            N(xp).red = false;
            if (xpp >= 0) {
              N(xpp).red = true;
              root = rotateRight(root, xpp);
            }
          }
        }
      } else {
        if (xppl >= 0 && N(xppl).red) {
          N(xppl).red = false;
          N(xp).red = false;
          N(xpp).red = true;
          x = xpp;
        } else {
          if (x == N(xp).left) {
            root = rotateRight(root, x = xp);
            xpp = (xp = N(x).parent) < 0 ? -1 : N(xp).parent;
          }
          if (xp >= 0) {
            N(xp).red = false;
            if (xpp >= 0) {
              N(xpp).red = true;
              root = rotateLeft(root, xpp);
            }
          }
        }
      }
    }
  }
  int balanceDeletion(int root, int x) {
    for (int xp, xpl, xpr;;) {
      if (x < 0 || x == root) {
        return root;
      } else if ((xp = N(x).parent) < 0) {
        N(x).red = false;
        return x;
      } else if (N(x).red) {
        N(x).red = false;
        return root;
      } else if ((xpl = N(xp).left) == x) {
        if ((xpr = N(xp).right) >= 0 && N(xpr).red) {
          N(xpr).red = false;
          N(xp).red = true;
          root = rotateLeft(root, xp);
          xpr = (xp = N(x).parent) < 0 ? -1 : N(xp).right;
        }
        if (xpr < 0) {
          x = xp;
        } else {
          const int sl = N(xpr).left;
          int sr = N(xpr).right;
          if ((sr < 0 || !N(sr).red) && (sl < 0 || !N(sl).red)) {
            N(xpr).red = true;
            x = xp;
          } else {
            if (sr < 0 || !N(sr).red) {
              if (sl >= 0) N(sl).red = false;
              N(xpr).red = true;
              root = rotateRight(root, xpr);
              xpr = (xp = N(x).parent) < 0 ? -1 : N(xp).right;
            }
            if (xpr >= 0) {
              N(xpr).red = (xp < 0) ? false : N(xp).red;
              if ((sr = N(xpr).right) >= 0) N(sr).red = false;
            }
            if (xp >= 0) {
              N(xp).red = false;
              root = rotateLeft(root, xp);
            }
            x = root;
          }
        }
      } else {  // symmetric
        if (xpl >= 0 && N(xpl).red) {
          N(xpl).red = false;
          N(xp).red = true;
          root = rotateRight(root, xp);
          xpl = (xp = N(x).parent) < 0 ? -1 : N(xp).left;
        }
        if (xpl < 0) {
          x = xp;
        } else {
          int sl = N(xpl).left;
          const int sr = N(xpl).right;
          if ((sl < 0 || !N(sl).red) && (sr < 0 || !N(sr).red)) {
            N(xpl).red = true;
            x = xp;
          } else {
            if (sl < 0 || !N(sl).red) {
              if (sr >= 0) N(sr).red = false;
              N(xpl).red = true;
              root = rotateLeft(root, xpl);
              xpl = (xp = N(x).parent) < 0 ? -1 : N(xp).left;
            }
            if (xpl >= 0) {
              N(xpl).red = (xp < 0) ? false : N(xp).red;
              if ((sl = N(xpl).left) >= 0) N(sl).red = false;
            }
            if (xp >= 0) {
              N(xp).red = false;
              root = rotateRight(root, xp);
            }
            x = root;
          }
        }
      }
    }
  }
};

}  // namespace oracle
