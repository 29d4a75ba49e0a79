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
// The tree is kept in a flat node array (index links) so an in-order snapshot for a device scan is one walk.
#pragma once
#include <algorithm>
#include <atomic>
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
// Nodes are one 20-byte record each (key, links, colour) so a search step is one cache line.
struct RbNode {
  uint32_t kc;  // key (a non-negative int) with the colour in bit 31
  union {
    struct {
      int left, right;
    };
    int ch[2];  // ch[0] = left, ch[1] = right: the build's fix-up picks a side by index instead of by branch
  };
  int parent;
  int key() const { return (int)(kc & 0x7fffffffu); }
  bool red() const { return (kc >> 31) != 0; }
  void setRed(bool r) { kc = (kc & 0x7fffffffu) | ((uint32_t)r << 31); }
  void setKey(int k) { kc = (kc & 0x80000000u) | (uint32_t)k; }
};
template <class Cmp>
class RbTreeSet {
  template <class>
  friend class RbTreeSet;

 public:
  explicit RbTreeSet(Cmp c) : cmp_(c) {}
  // Take over the structure (nodes, colours, in-order sequence) of a tree built elsewhere, e.g. by buildByRank on a
  // helper thread; `o` is left with this tree's old structure.
  template <class C2>
  void adopt(RbTreeSet<C2>& o) {
    n_.swap(o.n_);
    free_.swap(o.free_);
    std::swap(root_, o.root_);
    std::swap(size_, o.size_);
    std::swap(seqOn_, o.seqOn_);
    seqId_.swap(o.seqId_);
    seqKey_.swap(o.seqKey_);
    building_ = o.building_ = false;
  }
  void clear() {
    building_ = false;
    n_.clear();
    free_.clear();
    root_ = -1;
    size_ = 0;
    seqOn_ = false;
    seqId_.clear();
    seqKey_.clear();
  }
  int size() const { return size_; }
  // diagnostics / tests: a fingerprint of the structure (keys with their links and colours, walked from the root)
  uint64_t shapeHash() const {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&h](int64_t v) { h = (h ^ (uint64_t)v) * 1099511628211ull; };
    std::vector<int> st;
    if (root_ >= 0) st.push_back(root_);
    while (!st.empty()) {
      const int p = st.back();
      st.pop_back();
      mix(n_[p].key());
      mix(n_[p].red());
      mix(n_[p].left >= 0 ? n_[n_[p].left].key() : -1);
      mix(n_[p].right >= 0 ? n_[n_[p].right].key() : -1);
      if (n_[p].right >= 0) st.push_back(n_[p].right);
      if (n_[p].left >= 0) st.push_back(n_[p].left);
    }
    return h;
  }
  bool add(int k) {
    int t = root_;
    if (t < 0) {
      root_ = alloc(k, -1);
      size_ = 1;
      if (seqOn_) {
        seqId_.assign(1, root_);
        seqKey_.assign(1, k);
      }
      return true;
    }
    int parent = -1, c = 0;
    while (t >= 0) {
      parent = t;
      c = cmp_(k, n_[t].key());
      if (c < 0) t = n_[t].left;
      else if (c > 0) t = n_[t].right;
      else return false;
    }
    int e = alloc(k, parent);
    (c < 0 ? n_[parent].left : n_[parent].right) = e;
    if (seqOn_) {  // a new leaf sits right before (left child) or after (right child) its parent in order
      const size_t at = seqPos(parent) + (c < 0 ? 0 : 1);
      seqId_.insert(seqId_.begin() + at, e);
      seqKey_.insert(seqKey_.begin() + at, k);
    }
    insertFix(e);
    ++size_;
    return true;
  }
  // Insert `ids` in order into an EMPTY tree whose comparator agrees with `rank` (distinct ranks in [0, n)) on
  // these elements: the same sequence of TreeMap.put calls and therefore the same structure. The search is not
  // walked: a put lands on the one empty link between the new key's in-order neighbours (the predecessor's right
  // link when that is empty, else the successor's left link), found in a two-level bitmap over the ranks. The node of
  // a key is its rank, so a put's parent is its in-order neighbour and the puts walk nearby nodes.
  // `cancel` (optional) stops the build early (the tree is then incomplete and must be discarded).
  void buildByRank(const std::vector<int>& ids, const std::vector<int32_t>& rank,
                   const std::atomic<bool>* cancel = nullptr) {
    std::vector<int> i2(ids);
    std::vector<int32_t> r2(rank);
    buildByRank(std::move(i2), std::move(r2), cancel);
  }
  // withSequence = false: the in-order sequence is not taken at the end (a tree that will only be searched)
  void buildByRank(std::vector<int>&& ids, std::vector<int32_t>&& rank, const std::atomic<bool>* cancel = nullptr,
                   bool withSequence = true) {
    buildStart(std::move(ids), std::move(rank), withSequence);
    while (!buildStep(512))
      if (cancel && cancel->load(std::memory_order_relaxed)) return;
  }
  // The same build a bounded number of puts at a time (buildStep returns true once every put is done, then the
  // tree is complete); the tree must not be used before.
  void buildStart(std::vector<int>&& ids, std::vector<int32_t>&& rank, bool withSequence = true) {
    bSeq_ = withSequence;
    free_.clear();
    root_ = -1;
    size_ = 0;
    bIds_ = std::move(ids);
    bRank_ = std::move(rank);
    bNext_ = 0;
    int32_t nr = 0;
    for (int k : bIds_) nr = std::max(nr, bRank_[k] + 1);
    bNr_ = nr;
    n_.resize(nr);  // every put writes its rank's node whole; ranks no id takes stay unused (never linked), so the
                    // slots kept from an earlier build are not cleared
    bW_.assign((nr + 63) >> 6, 0);
    bSw_.assign((bW_.size() + 63) >> 6, 0);
    seqOn_ = false;
    building_ = true;
  }
  bool buildStep(size_t maxPuts) {
    if (!building_) return true;
    Node* N = n_.data();
    const size_t end = maxPuts >= bIds_.size() - bNext_ ? bIds_.size() : bNext_ + maxPuts;
    for (size_t e = bNext_; e < end; ++e) {
      const int k = bIds_[e];
      const int32_t rk = bRank_[k];
#ifndef CCMI_TREE_PF
#define CCMI_TREE_PF 0
#endif
#if CCMI_TREE_PF > 0
      if (e + CCMI_TREE_PF < bIds_.size()) {  // a later put's node and in-order neighbours into cache ahead of its turn
        const int32_t r2 = bRank_[bIds_[e + CCMI_TREE_PF]];
        __builtin_prefetch(&N[r2], 1, 3);
        const int32_t p2 = bPred(r2), s2 = bSucc(r2);
        if (p2 >= 0) __builtin_prefetch(&N[p2], 1, 3);
        if (s2 >= 0) __builtin_prefetch(&N[s2], 1, 3);
      }
#endif
      if (e == 0) {
        N[rk] = Node{(uint32_t)k, -1, -1, -1};
        root_ = rk;
        size_ = 1;
      } else {
        // the empty link between the in-order neighbours: the predecessor's right one when free, else the successor's left
        const int32_t pr = bPred(rk), sc = bSucc(rk);
        const int side = pr >= 0 && N[pr].right < 0 ? 1 : 0;
        const int parent = side ? pr : sc;
        N[rk] = Node{(uint32_t)k, {{-1, -1}}, parent};
        N[parent].ch[side] = rk;
        insertFixDir(N, rk);
        ++size_;
      }
      bW_[rk >> 6] |= 1ull << (rk & 63);
      bSw_[rk >> 12] |= 1ull << ((rk >> 6) & 63);
    }
    bNext_ = end;
    if (bNext_ < bIds_.size()) return false;
    building_ = false;
    if (!bSeq_) {
      seqOn_ = false;
      seqId_.clear();
      seqKey_.clear();
      return true;
    }
    // from here on the in-order sequence is maintained next to the tree (rotations do not change it)
    seqId_.clear();
    for (size_t wi = 0; wi < bW_.size(); ++wi)
      for (uint64_t m = bW_[wi]; m; m &= m - 1) seqId_.push_back((int)((wi << 6) | __builtin_ctzll(m)));
    seqKey_.resize(seqId_.size());
    for (size_t i = 0; i < seqId_.size(); ++i) seqKey_[i] = n_[seqId_[i]].key();
    seqOn_ = true;
    building_ = false;
    return true;
  }
  bool building() const { return building_; }
  // Stop maintaining the in-order sequence (trees that are only searched: add/remove then skip its O(n) updates)
  void untrackSequence() {
    seqOn_ = false;
    seqId_.clear();
    seqKey_.clear();
  }
  // Maintain the in-order sequence next to the tree from now on (a tree built by add(): one traversal), so
  // inorder() is a copy instead of a walk over every node.
  void trackSequence() {
    if (seqOn_) return;
    seqId_.clear();
    int p = root_;
    if (p >= 0) {
      while (n_[p].left >= 0) p = n_[p].left;
      for (; p >= 0; p = succ(p)) seqId_.push_back(p);
    }
    seqKey_.resize(seqId_.size());
    for (size_t i = 0; i < seqId_.size(); ++i) seqKey_[i] = n_[seqId_[i]].key();
    seqOn_ = true;
  }
  bool remove(int k) {
    int p = find(k);
    if (p < 0) return false;
    erase(p);
    return true;
  }
  bool contains(int k) const { return find(k) >= 0; }
  // Collection.removeIf over the TreeSet iterator: no comparator, so stale nodes are found too. TreeMap's
  // PrivateEntryIterator.remove continues at the removed entry when it had two children (deleteEntry moved its
  // successor's key in), which is the same in-order position of the sequence either way.
  template <class Pred>
  bool removeIf(Pred pred) {
    bool removed = false;
    if (seqOn_) {
      for (size_t i = 0; i < seqKey_.size();) {
        if (pred(seqKey_[i])) {
          erase(seqId_[i]);
          removed = true;
        } else {
          ++i;
        }
      }
      return removed;
    }
    int p = root_;
    if (p < 0) return false;
    while (n_[p].left >= 0) p = n_[p].left;
    while (p >= 0) {
      int next = succ(p);
      if (pred(n_[p].key())) {
        if (n_[p].left >= 0 && n_[p].right >= 0) next = p;
        erase(p);
        removed = true;
      }
      p = next;
    }
    return removed;
  }
  // the maintained in-order key sequence (no copy), or null when it is not maintained; valid until the next change
  const std::vector<int>* sequence() const { return seqOn_ ? &seqKey_ : nullptr; }
  void inorder(std::vector<int>& out) const {
    if (seqOn_) {
      out.assign(seqKey_.begin(), seqKey_.end());
      return;
    }
    out.clear();
    int p = root_;
    if (p < 0) return;
    while (n_[p].left >= 0) p = n_[p].left;
    for (; p >= 0; p = succ(p)) out.push_back(n_[p].key());
  }

 private:
  using Node = RbNode;
  Cmp cmp_;
  std::vector<Node> n_;
  std::vector<int> free_;
  int root_ = -1, size_ = 0;
  bool seqOn_ = false;
  std::vector<int> seqId_, seqKey_;  // node ids / keys in order (after buildByRank)
  // a build in progress (buildStart / buildStep): the put sequence, the next put, the two-level bitmap of put ranks
  bool building_ = false, bSeq_ = true;
  std::vector<int> bIds_;
  std::vector<int32_t> bRank_;
  size_t bNext_ = 0;
  int32_t bNr_ = 0;
  std::vector<uint64_t> bW_, bSw_;
  int32_t bPred(int32_t r) const {  // largest put rank < r, or -1
    int wi = r >> 6;
    uint64_t m = bW_[wi] & ((1ull << (r & 63)) - 1);
    if (m) return (wi << 6) | (63 - __builtin_clzll(m));
    int si = wi >> 6;
    uint64_t sm = bSw_[si] & ((1ull << (wi & 63)) - 1);
    while (!sm) {
      if (--si < 0) return -1;
      sm = bSw_[si];
    }
    wi = (si << 6) | (63 - __builtin_clzll(sm));
    return (wi << 6) | (63 - __builtin_clzll(bW_[wi]));
  }
  int32_t bSucc(int32_t r) const {  // smallest put rank > r, or -1
    const int ns = (int)bSw_.size();
    int wi = r >> 6;
    uint64_t m = (r & 63) == 63 ? 0 : bW_[wi] & (~0ull << ((r & 63) + 1));
    if (m) return (wi << 6) | __builtin_ctzll(m);
    int si = wi >> 6;
    uint64_t sm = (wi & 63) == 63 ? 0 : bSw_[si] & (~0ull << ((wi & 63) + 1));
    while (!sm) {
      if (++si >= ns) return -1;
      sm = bSw_[si];
    }
    wi = (si << 6) | __builtin_ctzll(sm);
    return (wi << 6) | __builtin_ctzll(bW_[wi]);
  }

  size_t seqPos(int node) const { return (size_t)(std::find(seqId_.begin(), seqId_.end(), node) - seqId_.begin()); }

  int alloc(int k, int parent) {
    int id;
    if (!free_.empty()) {
      id = free_.back();
      free_.pop_back();
      n_[id] = Node{(uint32_t)k, -1, -1, parent};
    } else {
      id = (int)n_.size();
      n_.push_back(Node{(uint32_t)k, -1, -1, parent});
    }
    return id;
  }
  int find(int k) const {
    int p = root_;
    while (p >= 0) {
      int c = cmp_(k, n_[p].key());
      if (c == 0) return p;
      p = c < 0 ? n_[p].left : n_[p].right;
    }
    return -1;
  }
  int succ(int t) const {
    if (n_[t].right >= 0) {
      int p = n_[t].right;
      while (n_[p].left >= 0) p = n_[p].left;
      return p;
    }
    int p = n_[t].parent, ch = t;
    while (p >= 0 && ch == n_[p].right) {
      ch = p;
      p = n_[p].parent;
    }
    return p;
  }
  bool isRed(int p) const { return p >= 0 && n_[p].red(); }
  int par(int p) const { return p < 0 ? -1 : n_[p].parent; }
  int lft(int p) const { return p < 0 ? -1 : n_[p].left; }
  int rgt(int p) const { return p < 0 ? -1 : n_[p].right; }
  void paint(int p, bool red) {
    if (p >= 0) n_[p].setRed(red);
  }
  void rotL(int p) {
    if (p < 0) return;
    Node& P = n_[p];
    const int r = P.right;
    Node& Rn = n_[r];
    P.right = Rn.left;
    if (Rn.left >= 0) n_[Rn.left].parent = p;
    Rn.parent = P.parent;
    if (P.parent < 0) root_ = r;
    else if (n_[P.parent].left == p) n_[P.parent].left = r;
    else n_[P.parent].right = r;
    Rn.left = p;
    P.parent = r;
  }
  void rotR(int p) {
    if (p < 0) return;
    Node& P = n_[p];
    const int l = P.left;
    Node& L = n_[l];
    P.left = L.right;
    if (L.right >= 0) n_[L.right].parent = p;
    L.parent = P.parent;
    if (P.parent < 0) root_ = l;
    else if (n_[P.parent].right == p) n_[P.parent].right = l;
    else n_[P.parent].left = l;
    L.right = p;
    P.parent = l;
  }
  // TreeMap.fixAfterInsertion (a red parent is never the root, so the grandparent exists; after the rotation case
  // the parent of x is black and the JDK loop ends)
  void insertFix(int x) {
    Node* N = n_.data();
    N[x].setRed(1);
    while (x != root_) {
      int p = N[x].parent;
      if (!N[p].red()) break;
      const int g = N[p].parent;
      if (p == N[g].left) {
        const int y = N[g].right;
        if (y >= 0 && N[y].red()) {
          N[p].setRed(0);
          N[y].setRed(0);
          N[g].setRed(1);
          x = g;
          continue;
        }
        if (x == N[p].right) {
          x = p;
          rotL(x);
          p = N[x].parent;
        }
        N[p].setRed(0);
        N[g].setRed(1);
        rotR(g);
      } else {
        const int y = N[g].left;
        if (y >= 0 && N[y].red()) {
          N[p].setRed(0);
          N[y].setRed(0);
          N[g].setRed(1);
          x = g;
          continue;
        }
        if (x == N[p].left) {
          x = p;
          rotR(x);
          p = N[x].parent;
        }
        N[p].setRed(0);
        N[g].setRed(1);
        rotL(g);
      }
      break;
    }
    N[root_].setRed(0);
  }
  // insertFix with the two mirrored cases folded by side index (d: the side of g that p hangs on), for the builds:
  // the same recolourings and rotations in the same order, fewer data-dependent branches
  void rotDir(Node* N, int p, int d) {  // rotate p down to side d: its child on side 1 - d takes its place
    const int c = N[p].ch[1 - d];
    const int cc = N[c].ch[d];
    N[p].ch[1 - d] = cc;
    if (cc >= 0) N[cc].parent = p;
    const int pp = N[p].parent;
    N[c].parent = pp;
    if (pp < 0) root_ = c;
    else N[pp].ch[N[pp].ch[1] == p ? 1 : 0] = c;
    N[c].ch[d] = p;
    N[p].parent = c;
  }
  void insertFixDir(Node* N, int x) {
    N[x].setRed(1);
    while (x != root_) {
      int p = N[x].parent;
      if (!N[p].red()) break;
      const int g = N[p].parent;
      const int d = N[g].ch[1] == p ? 1 : 0;
      const int y = N[g].ch[1 - d];
      if (y >= 0 && N[y].red()) {
        N[p].setRed(0);
        N[y].setRed(0);
        N[g].setRed(1);
        x = g;
        continue;
      }
      if (x == N[p].ch[1 - d]) {  // the inner grandchild: p rotates down to side d first
        x = p;
        rotDir(N, x, d);
        p = N[x].parent;
      }
      N[p].setRed(0);
      N[g].setRed(1);
      rotDir(N, g, 1 - d);
      break;
    }
    N[root_].setRed(0);
  }
  // TreeMap.deleteEntry (successor key copied into the doomed node) + fixAfterDeletion
  void erase(int p) {
    --size_;
    if (seqOn_) {  // the doomed key leaves the sequence at p's position (p takes its successor's key below)
      const size_t at = seqPos(p);
      if (n_[p].left >= 0 && n_[p].right >= 0) {
        seqKey_[at] = seqKey_[at + 1];
        seqId_.erase(seqId_.begin() + at + 1);
        seqKey_.erase(seqKey_.begin() + at + 1);
      } else {
        seqId_.erase(seqId_.begin() + at);
        seqKey_.erase(seqKey_.begin() + at);
      }
    }
    if (n_[p].left >= 0 && n_[p].right >= 0) {
      int s = succ(p);
      n_[p].setKey(n_[s].key());
      p = s;
    }
    int rep = n_[p].left >= 0 ? n_[p].left : n_[p].right;
    if (rep >= 0) {
      const int pp = n_[p].parent;
      n_[rep].parent = pp;
      if (pp < 0) root_ = rep;
      else if (p == n_[pp].left) n_[pp].left = rep;
      else n_[pp].right = rep;
      n_[p].left = n_[p].right = n_[p].parent = -1;
      if (!n_[p].red()) deleteFix(rep);
    } else if (n_[p].parent < 0) {
      root_ = -1;
    } else {
      if (!n_[p].red()) deleteFix(p);
      int pp = n_[p].parent;
      if (pp >= 0) {
        if (p == n_[pp].left) n_[pp].left = -1;
        else if (p == n_[pp].right) n_[pp].right = -1;
        n_[p].parent = -1;
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
  // The k-th element of the sorted run after the poll position (-1 past its end): a likely future poll (elements
  // re-added through the heap are not included)
  int upcoming(size_t k) const { return pos_ + k < s_.size() ? s_[pos_ + k] : -1; }
  // The sorted run's elements not yet polled (in poll order while the heap is empty), and skipping k of them: the
  // same as k polls when the heap is empty
  bool heapEmpty() const { return heap_.empty(); }
  // the heap's next element and its poll; the sorted run's elements (from the poll position) that poll before x
  int heapPeek() const { return heap_.peek(); }
  int heapPoll() { return heap_.poll(); }
  size_t runBefore(int x) const {
    const auto b = s_.begin() + (ptrdiff_t)std::min(pos_, s_.size());
    return (size_t)(std::partition_point(b, s_.end(), [&](int y) { return cmp_(x, y) >= 0; }) - b);
  }
  const int* runData() const { return s_.data() + pos_; }
  size_t runLeft() const { return pos_ < s_.size() ? s_.size() - pos_ : 0; }
  void skipRun(size_t k) { pos_ += k; }
  // Put back the most recently polled element (un-polls come in reverse poll order). An element that came from
  // the sorted run and whose key did not change since returns to its slot in the run (O(1)); anything else goes
  // through the heap. Either way the queue holds the same set, so the poll order is unchanged.
  void unpoll(int x) {
    if (pos_ > 0 && s_[pos_ - 1] == x) --pos_;
    else heap_.add(x);
  }

 private:
  Cmp cmp_;
  JavaPQ<Cmp> heap_;
  std::vector<int> s_;
  size_t pos_ = 0;
};

// Iteration order of a HashSet<Broker> filled by add() in `ins` order (Broker.hashCode() == id).
// HashSet<Broker> table capacity after n distinct add() calls from the default table (16 buckets, load .75)
inline uint32_t javaHashSetCapacity(size_t n) {
  uint32_t cap = 16;
  while (n > (size_t)(cap / 4 * 3)) cap <<= 1;
  return cap;
}

inline void javaHashSetOrder(const std::vector<int>& ins, std::vector<int>& out) {
  auto slot = [](int h, unsigned c) { return (unsigned)(h ^ (int)((unsigned)h >> 16)) & (c - 1); };
  if (ins.size() <= 8) {  // the default 16-bucket table never resizes or treeifies: bucket order, insertion order within
    int ks[8];
    unsigned sl[8];
    int m = 0;
    for (int k : ins) {
      bool dup = false;
      for (int i = 0; i < m; ++i) dup |= ks[i] == k;
      if (dup) continue;
      int j = m++;
      const unsigned s0 = slot(k, 16);
      while (j > 0 && sl[j - 1] > s0) {
        ks[j] = ks[j - 1];
        sl[j] = sl[j - 1];
        --j;
      }
      ks[j] = k;
      sl[j] = s0;
    }
    out.assign(ks, ks + m);
    return;
  }
  const size_t N = ins.size();
  {
    // Strictly ascending non-negative keys below both the final table capacity and 2^16 (where the hash spread is the
    // identity): every key ends in a bucket of its own, whatever resizes or tree bins happened on the way, so the
    // iteration order is the keys' ascending order — the input itself.
    bool asc = ins.front() >= 0;
    for (size_t i = 1; i < N && asc; ++i) asc = ins[i - 1] < ins[i];
    if (asc && (size_t)ins.back() < std::min<size_t>(javaHashSetCapacity(N), 65536)) {
      out.assign(ins.begin(), ins.end());
      return;
    }
  }
  // General case: the JDK 11 HashMap insertion (bucket lists appended at the tail; a resize splits every list in
  // order, so each bucket keeps insertion order; a list reaching 9 nodes resizes a table below 64 buckets), on flat
  // arrays.
  unsigned cap = 16;
  std::vector<int> key(N), nxt(N), head(cap, -1), tail(cap, -1), cnt(cap, 0);
  size_t n = 0;
  auto rehash = [&]() {
    const unsigned nc = cap << 1;
    std::vector<int> nh(nc, -1), nt(nc, -1), nn(nc, 0);
    for (unsigned b = 0; b < cap; ++b)
      for (int e = head[b]; e >= 0;) {
        const int following = nxt[e];
        const unsigned t = slot(key[e], nc);
        nxt[e] = -1;
        if (nt[t] < 0) nh[t] = e;
        else nxt[nt[t]] = e;
        nt[t] = e;
        nn[t]++;
        e = following;
      }
    head.swap(nh);
    tail.swap(nt);
    cnt.swap(nn);
    cap = nc;
  };
  for (int k : ins) {
    const unsigned b = slot(k, cap);
    bool dup = false;
    for (int e = head[b]; e >= 0 && !dup; e = nxt[e]) dup = key[e] == k;
    if (dup) continue;
    const int e = (int)n;
    key[e] = k;
    nxt[e] = -1;
    if (tail[b] < 0) head[b] = e;
    else nxt[tail[b]] = e;
    tail[b] = e;
    if (++cnt[b] >= 9) {
      if (cap < 64) rehash();
      else throw std::runtime_error("HashSet tree bin order is not emulated");
    }
    if (++n > (size_t)(cap * 3 / 4)) rehash();
  }
  out.clear();
  out.reserve(n);
  for (unsigned b = 0; b < cap; ++b)
    for (int e = head[b]; e >= 0; e = nxt[e]) out.push_back(key[e]);
}

// ((Double) x).intValue() / (int) x: NaN -> 0, saturating, truncation toward zero (JLS 5.1.3)
inline int32_t jD2I(double x) {
  if (x != x) return 0;
  if (x >= 2147483647.0) return 2147483647;
  if (x <= -2147483648.0) return (int32_t)0x80000000;
  return (int32_t)x;
}
inline int32_t jAddI(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }  // Java int + (wraps)
inline int32_t jSubI(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }

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
