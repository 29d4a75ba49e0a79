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
#include <algorithm>
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

inline int32_t jStringHash(const char* s) {  // String.hashCode
  uint32_t h = 0;
  for (; *s; ++s) h = 31u * h + (uint32_t)(unsigned char)*s;
  return (int32_t)h;
}
inline int32_t jMix(int32_t h, int32_t x) { return (int32_t)(31u * (uint32_t)h + (uint32_t)x); }  // Objects.hash step

// ----------------------------------------------------------------------------------------------
// java.util.HashSet<E> (JDK 11 HashMap<E, PRESENT>) over elements named by an int id. The iteration order of
// a HashSet leaks into several goal drivers (Broker.replicas(), new HashSet<>(broker.leaderReplicas()),
// Broker.topics(), Broker.currentOfflineReplicas()), so the table is emulated
// operation for operation: spread hash h ^ (h >>> 16), power-of-two buckets, list bins in insertion order,
// order-preserving resize splits, bins of more than 8 nodes turned into red-black TreeNode bins (or a resize
// below 64 buckets), TreeNode insertion after its tree parent in the next-chain, root moved to the front,
// removeTreeNode with successor swap and untreeify of small trees, TreeNode.split on resize.
// Elements with equal hashes are ordered by Ops::cmp (E implements Comparable<E>); distinct elements never
// compare equal, so tieBreakOrder is never reached.
//   Ops: int cmp(int a, int b) const
template <class Ops>
class JHashSet {
 public:
  explicit JHashSet(const Ops* ops = nullptr) : ops_(ops) {}
  void setOps(const Ops* ops) { ops_ = ops; }
  int size() const { return size_; }
  // HashSet(Collection c): HashMap(max((int)(c.size() / .75f) + 1, 16)), then c's elements in c's order
  void assignCopy(const JHashSet& src) {
    clearAll();
    ops_ = src.ops_;
    threshold_ = tableSizeFor(std::max((int)((float)src.size() / 0.75f) + 1, 16));
    for (int head : src.tab_)
      for (int e = head; e >= 0; e = src.nd_[e].next) add(src.nd_[e].id, src.nd_[e].hash, true);
  }
  bool add(int id, int32_t hashCode) { return add(id, spread(hashCode), true); }
  bool remove(int id, int32_t hashCode) {
    if (tab_.empty()) return false;
    const int32_t h = spread(hashCode);
    const int i = ((int)tab_.size() - 1) & h;
    const int first = tab_[i];
    if (first < 0) return false;
    int node = -1;
    if (nd_[first].tree) {
      node = find(root(first), h, id);
      if (node < 0) return false;
      removeTreeNode(node);
    } else {
      int prev = -1;
      for (int e = first; e >= 0; prev = e, e = nd_[e].next)
        if (nd_[e].hash == h && nd_[e].id == id) {
          node = e;
          break;
        }
      if (node < 0) return false;
      if (prev < 0) tab_[i] = nd_[node].next;
      else nd_[prev].next = nd_[node].next;
    }
    free_.push_back(node);
    --size_;
    return true;
  }
  template <class F>
  void forEach(F f) const {
    for (int head : tab_)
      for (int e = head; e >= 0; e = nd_[e].next) f(nd_[e].id);
  }
  void order(std::vector<int32_t>& out) const {
    out.clear();
    forEach([&](int id) { out.push_back(id); });
  }

 private:
  struct Node {
    int id;
    int32_t hash;
    int next, prev, parent, left, right;
    bool red, tree;
  };
  const Ops* ops_;
  std::vector<Node> nd_;
  std::vector<int> free_, tab_;
  int size_ = 0, threshold_ = 0;

  static int32_t spread(int32_t h) { return h ^ (int32_t)((uint32_t)h >> 16); }
  static int tableSizeFor(int c) {
    int n = 1;
    while (n < c) n <<= 1;
    return n;
  }
  void clearAll() {
    nd_.clear();
    free_.clear();
    tab_.clear();
    size_ = threshold_ = 0;
  }
  int cmp(int a, int b) const { return ops_ ? ops_->cmp(a, b) : 0; }
  int alloc(int id, int32_t h, int next) {
    int k;
    if (!free_.empty()) {
      k = free_.back();
      free_.pop_back();
    } else {
      k = (int)nd_.size();
      nd_.emplace_back();
    }
    nd_[k] = Node{id, h, next, -1, -1, -1, -1, false, false};
    return k;
  }
  // HashMap.putVal (h already spread)
  bool add(int id, int32_t h, bool) {
    if (tab_.empty()) resize();
    const int i = ((int)tab_.size() - 1) & h;
    int p = tab_[i];
    if (p < 0) {
      tab_[i] = alloc(id, h, -1);
    } else if (nd_[p].tree) {
      if (!putTreeVal(i, id, h)) return false;
    } else {
      for (int bin = 0;; ++bin) {
        if (nd_[p].hash == h && nd_[p].id == id) return false;
        const int e = nd_[p].next;
        if (e < 0) {
          nd_[p].next = alloc(id, h, -1);
          if (bin >= 7) treeifyBin(h);
          break;
        }
        p = e;
      }
    }
    if (++size_ > threshold_) resize();
    return true;
  }
  void resize() {
    const int oldCap = (int)tab_.size();
    int newCap;
    if (oldCap > 0) {
      newCap = oldCap << 1;
      threshold_ = oldCap >= 16 ? threshold_ << 1 : (int)((float)newCap * 0.75f);
    } else if (threshold_ > 0) {
      newCap = threshold_;
      threshold_ = (int)((float)newCap * 0.75f);
    } else {
      newCap = 16;
      threshold_ = 12;
    }
    std::vector<int> old(newCap, -1);
    old.swap(tab_);
    for (int j = 0; j < oldCap; ++j) {
      const int e = old[j];
      if (e < 0) continue;
      if (nd_[e].next < 0) tab_[nd_[e].hash & (newCap - 1)] = e;
      else if (nd_[e].tree) split(e, j, oldCap);
      else splitList(e, j, oldCap);
    }
  }
  void splitList(int e, int j, int bit) {
    int loH = -1, loT = -1, hiH = -1, hiT = -1;
    for (int next; e >= 0; e = next) {
      next = nd_[e].next;
      int &H = (nd_[e].hash & bit) ? hiH : loH, &Tl = (nd_[e].hash & bit) ? hiT : loT;
      if (Tl < 0) H = e;
      else nd_[Tl].next = e;
      Tl = e;
    }
    if (loT >= 0) {
      nd_[loT].next = -1;
      tab_[j] = loH;
    }
    if (hiT >= 0) {
      nd_[hiT].next = -1;
      tab_[j + bit] = hiH;
    }
  }
  void treeifyBin(int32_t h) {
    const int n = (int)tab_.size();
    if (n < 64) {
      resize();
      return;
    }
    const int hd = tab_[(n - 1) & h];
    int tl = -1;
    for (int e = hd; e >= 0; e = nd_[e].next) {
      nd_[e].tree = true;
      nd_[e].prev = tl;
      tl = e;
    }
    if (hd >= 0) treeify(hd);
  }
  int dirOf(int32_t h, int id, int p) const {
    if (nd_[p].hash > h) return -1;
    if (nd_[p].hash < h) return 1;
    return cmp(id, nd_[p].id) <= 0 ? -1 : 1;
  }
  void treeify(int head) {
    int rt = -1;
    for (int x = head, next; x >= 0; x = next) {
      next = nd_[x].next;
      nd_[x].left = nd_[x].right = -1;
      if (rt < 0) {
        nd_[x].parent = -1;
        nd_[x].red = false;
        rt = x;
        continue;
      }
      for (int p = rt;;) {
        const int dir = dirOf(nd_[x].hash, nd_[x].id, p);
        const int xp = p;
        p = dir <= 0 ? nd_[p].left : nd_[p].right;
        if (p < 0) {
          nd_[x].parent = xp;
          (dir <= 0 ? nd_[xp].left : nd_[xp].right) = x;
          rt = balanceInsertion(rt, x);
          break;
        }
      }
    }
    moveRootToFront(rt);
  }
  void untreeify(int head) {
    for (int e = head; e >= 0; e = nd_[e].next) {
      nd_[e].tree = nd_[e].red = false;
      nd_[e].parent = nd_[e].left = nd_[e].right = nd_[e].prev = -1;
    }
  }
  int root(int p) const {
    while (nd_[p].parent >= 0) p = nd_[p].parent;
    return p;
  }
  void moveRootToFront(int rt) {
    if (rt < 0 || tab_.empty()) return;
    const int idx = ((int)tab_.size() - 1) & nd_[rt].hash;
    const int first = tab_[idx];
    if (rt == first) return;
    tab_[idx] = rt;
    const int rp = nd_[rt].prev, rn = nd_[rt].next;
    if (rn >= 0) nd_[rn].prev = rp;
    if (rp >= 0) nd_[rp].next = rn;
    if (first >= 0) nd_[first].prev = rt;
    nd_[rt].next = first;
    nd_[rt].prev = -1;
  }
  int find(int p, int32_t h, int id) const {  // TreeNode.find
    while (p >= 0) {
      const int pl = nd_[p].left, pr = nd_[p].right;
      if (nd_[p].hash > h) p = pl;
      else if (nd_[p].hash < h) p = pr;
      else if (nd_[p].id == id) return p;
      else if (pl < 0) p = pr;
      else if (pr < 0) p = pl;
      else {
        const int d = cmp(id, nd_[p].id);
        if (d != 0) {
          p = d < 0 ? pl : pr;
        } else {
          const int q = find(pr, h, id);
          if (q >= 0) return q;
          p = pl;
        }
      }
    }
    return -1;
  }
  bool putTreeVal(int i, int id, int32_t h) {  // false: already present
    const int rt = root(tab_[i]);
    bool searched = false;
    for (int p = rt;;) {
      int dir;
      if (nd_[p].hash > h) dir = -1;
      else if (nd_[p].hash < h) dir = 1;
      else if (nd_[p].id == id) return false;
      else if ((dir = cmp(id, nd_[p].id)) == 0) {
        if (!searched) {
          searched = true;
          if ((nd_[p].left >= 0 && find(nd_[p].left, h, id) >= 0) ||
              (nd_[p].right >= 0 && find(nd_[p].right, h, id) >= 0))
            return false;
        }
        throw std::runtime_error("HashMap.tieBreakOrder (identity hash order) cannot be reproduced");
      }
      const int xp = p;
      p = dir <= 0 ? nd_[p].left : nd_[p].right;
      if (p < 0) {
        const int xpn = nd_[xp].next;
        const int x = alloc(id, h, xpn);
        nd_[x].tree = true;
        (dir <= 0 ? nd_[xp].left : nd_[xp].right) = x;
        nd_[xp].next = x;
        nd_[x].parent = nd_[x].prev = xp;
        if (xpn >= 0) nd_[xpn].prev = x;
        moveRootToFront(balanceInsertion(rt, x));
        return true;
      }
    }
  }
  void removeTreeNode(int p) {
    const int idx = ((int)tab_.size() - 1) & nd_[p].hash;
    int first = tab_[idx], rt = first;
    const int succ = nd_[p].next, pred = nd_[p].prev;
    if (pred < 0) tab_[idx] = first = succ;
    else nd_[pred].next = succ;
    if (succ >= 0) nd_[succ].prev = pred;
    if (first < 0) return;
    if (nd_[rt].parent >= 0) rt = root(rt);
    int rl;
    if (nd_[rt].right < 0 || (rl = nd_[rt].left) < 0 || nd_[rl].left < 0) {
      untreeify(first);  // too small
      return;
    }
    const int pl = nd_[p].left, pr = nd_[p].right;
    int repl;
    if (pl >= 0 && pr >= 0) {
      int s = pr;
      while (nd_[s].left >= 0) s = nd_[s].left;
      std::swap(nd_[s].red, nd_[p].red);
      const int sr = nd_[s].right, pp = nd_[p].parent;
      if (s == pr) {
        nd_[p].parent = s;
        nd_[s].right = p;
      } else {
        const int sp = nd_[s].parent;
        if ((nd_[p].parent = sp) >= 0) (s == nd_[sp].left ? nd_[sp].left : nd_[sp].right) = p;
        if ((nd_[s].right = pr) >= 0) nd_[pr].parent = s;
      }
      nd_[p].left = -1;
      if ((nd_[p].right = sr) >= 0) nd_[sr].parent = p;
      if ((nd_[s].left = pl) >= 0) nd_[pl].parent = s;
      if ((nd_[s].parent = pp) < 0) rt = s;
      else (p == nd_[pp].left ? nd_[pp].left : nd_[pp].right) = s;
      repl = sr >= 0 ? sr : p;
    } else {
      repl = pl >= 0 ? pl : (pr >= 0 ? pr : p);
    }
    if (repl != p) {
      const int pp = nd_[repl].parent = nd_[p].parent;
      if (pp < 0) {
        rt = repl;
        nd_[repl].red = false;
      } else {
        (p == nd_[pp].left ? nd_[pp].left : nd_[pp].right) = repl;
      }
      nd_[p].left = nd_[p].right = nd_[p].parent = -1;
    }
    const int r = nd_[p].red ? rt : balanceDeletion(rt, repl);
    if (repl == p) {
      const int pp = nd_[p].parent;
      nd_[p].parent = -1;
      if (pp >= 0) {
        if (p == nd_[pp].left) nd_[pp].left = -1;
        else if (p == nd_[pp].right) nd_[pp].right = -1;
      }
    }
    moveRootToFront(r);
  }
  void split(int b, int idx, int bit) {  // TreeNode.split
    int loH = -1, loT = -1, hiH = -1, hiT = -1, lc = 0, hc = 0;
    for (int e = b, next; e >= 0; e = next) {
      next = nd_[e].next;
      nd_[e].next = -1;
      const bool hi = (nd_[e].hash & bit) != 0;
      int &H = hi ? hiH : loH, &Tl = hi ? hiT : loT;
      if ((nd_[e].prev = Tl) < 0) H = e;
      else nd_[Tl].next = e;
      Tl = e;
      ++(hi ? hc : lc);
    }
    if (loH >= 0) {
      tab_[idx] = loH;
      if (lc <= 6) untreeify(loH);
      else if (hiH >= 0) treeify(loH);
    }
    if (hiH >= 0) {
      tab_[idx + bit] = hiH;
      if (hc <= 6) untreeify(hiH);
      else if (loH >= 0) treeify(hiH);
    }
  }
  int rotateLeft(int rt, int p) {
    int r;
    if (p >= 0 && (r = nd_[p].right) >= 0) {
      const int rl = nd_[p].right = nd_[r].left;
      if (rl >= 0) nd_[rl].parent = p;
      const int pp = nd_[r].parent = nd_[p].parent;
      if (pp < 0) {
        rt = r;
        nd_[r].red = false;
      } else {
        (nd_[pp].left == p ? nd_[pp].left : nd_[pp].right) = r;
      }
      nd_[r].left = p;
      nd_[p].parent = r;
    }
    return rt;
  }
  int rotateRight(int rt, int p) {
    int l;
    if (p >= 0 && (l = nd_[p].left) >= 0) {
      const int lr = nd_[p].left = nd_[l].right;
      if (lr >= 0) nd_[lr].parent = p;
      const int pp = nd_[l].parent = nd_[p].parent;
      if (pp < 0) {
        rt = l;
        nd_[l].red = false;
      } else {
        (nd_[pp].right == p ? nd_[pp].right : nd_[pp].left) = l;
      }
      nd_[l].right = p;
      nd_[p].parent = l;
    }
    return rt;
  }
  bool red(int x) const { return x >= 0 && nd_[x].red; }
  int balanceInsertion(int rt, int x) {
    nd_[x].red = true;
    for (;;) {
      int xp = nd_[x].parent, xpp;
      if (xp < 0) {
        nd_[x].red = false;
        return x;
      }
      if (!nd_[xp].red || (xpp = nd_[xp].parent) < 0) return rt;
      const int xppl = nd_[xpp].left;
      if (xp == xppl) {
        const int xppr = nd_[xpp].right;
        if (red(xppr)) {
          nd_[xppr].red = nd_[xp].red = false;
          nd_[xpp].red = true;
          x = xpp;
        } else {
          if (x == nd_[xp].right) {
            rt = rotateLeft(rt, x = xp);
            xp = nd_[x].parent;
            xpp = xp < 0 ? -1 : nd_[xp].parent;
          }
          if (xp >= 0) {
            nd_[xp].red = false;
            if (xpp >= 0) {
              nd_[xpp].red = true;
              rt = rotateRight(rt, xpp);
            }
          }
        }
      } else {
        if (red(xppl)) {
          nd_[xppl].red = nd_[xp].red = false;
          nd_[xpp].red = true;
          x = xpp;
        } else {
          if (x == nd_[xp].left) {
            rt = rotateRight(rt, x = xp);
            xp = nd_[x].parent;
            xpp = xp < 0 ? -1 : nd_[xp].parent;
          }
          if (xp >= 0) {
            nd_[xp].red = false;
            if (xpp >= 0) {
              nd_[xpp].red = true;
              rt = rotateLeft(rt, xpp);
            }
          }
        }
      }
    }
  }
  int balanceDeletion(int rt, int x) {
    for (;;) {
      int xp;
      if (x < 0 || x == rt) return rt;
      if ((xp = nd_[x].parent) < 0) {
        nd_[x].red = false;
        return x;
      }
      if (nd_[x].red) {
        nd_[x].red = false;
        return rt;
      }
      if (nd_[xp].left == x) {
        int xpr = nd_[xp].right;
        if (red(xpr)) {
          nd_[xpr].red = false;
          nd_[xp].red = true;
          rt = rotateLeft(rt, xp);
          xp = nd_[x].parent;
          xpr = xp < 0 ? -1 : nd_[xp].right;
        }
        if (xpr < 0) {
          x = xp;
          continue;
        }
        int sl = nd_[xpr].left, sr = nd_[xpr].right;
        if (!red(sr) && !red(sl)) {
          nd_[xpr].red = true;
          x = xp;
          continue;
        }
        if (!red(sr)) {
          if (sl >= 0) nd_[sl].red = false;
          nd_[xpr].red = true;
          rt = rotateRight(rt, xpr);
          xp = nd_[x].parent;
          xpr = xp < 0 ? -1 : nd_[xp].right;
        }
        if (xpr >= 0) {
          nd_[xpr].red = xp < 0 ? false : nd_[xp].red;
          if ((sr = nd_[xpr].right) >= 0) nd_[sr].red = false;
        }
        if (xp >= 0) {
          nd_[xp].red = false;
          rt = rotateLeft(rt, xp);
        }
        x = rt;
      } else {
        int xpl = nd_[xp].left;
        if (red(xpl)) {
          nd_[xpl].red = false;
          nd_[xp].red = true;
          rt = rotateRight(rt, xp);
          xp = nd_[x].parent;
          xpl = xp < 0 ? -1 : nd_[xp].left;
        }
        if (xpl < 0) {
          x = xp;
          continue;
        }
        int sl = nd_[xpl].left, sr = nd_[xpl].right;
        if (!red(sl) && !red(sr)) {
          nd_[xpl].red = true;
          x = xp;
          continue;
        }
        if (!red(sl)) {
          if (sr >= 0) nd_[sr].red = false;
          nd_[xpl].red = true;
          rt = rotateLeft(rt, xpl);
          xp = nd_[x].parent;
          xpl = xp < 0 ? -1 : nd_[xp].left;
        }
        if (xpl >= 0) {
          nd_[xpl].red = xp < 0 ? false : nd_[xp].red;
          if ((sl = nd_[xpl].left) >= 0) nd_[sl].red = false;
        }
        if (xp >= 0) {
          nd_[xp].red = false;
          rt = rotateRight(rt, xp);
        }
        x = rt;
      }
    }
  }
};

// DoubleStream.sum() of JDK 11 (Collectors.sumWithCompensation, computeFinalSum): Kahan summation plus the
// simple sum for the infinite/NaN case.
struct JDoubleSum {
  double s0 = 0, s1 = 0, simple = 0;
  void add(double v) {
    simple += v;
    const double y = v - s1, t = s0 + y;
    s1 = (t - s0) - y;
    s0 = t;
  }
  double result() const {
    const double tmp = s0 + s1;
    return (std::isnan(tmp) && std::isinf(simple)) ? simple : tmp;
  }
};

}  // namespace ccmi
