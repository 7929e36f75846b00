#include "huffman.hpp"

#include <algorithm>
#include <climits>
#include <cstdint>
#include <memory>
#include <numeric>
#include <queue>
#include <unordered_map>

namespace jpge {
namespace {

constexpr int kLimit = 15;  // package_merge(symbols, 15), Huffman.cpp:29

// A heap entry.  Only `weight` takes part in comparisons, exactly like the
// reference's Package comparator (Huffman.hpp:117-119), so std::priority_queue
// performs the identical permutation sequence whatever the payload is.
struct Item {
    int weight;
    int node;
};
struct ItemGreater {
    bool operator()(const Item& a, const Item& b) const { return a.weight > b.weight; }
};
using Level = std::priority_queue<Item, std::vector<Item>, ItemGreater>;

}  // namespace

void build_code_lengths_std(const std::vector<std::pair<int, int>>& first_order_counts,
                            std::vector<std::vector<int>>& by_len) {
    // symbol_counts (Huffman.cpp:6-9): insertion in first-occurrence order; the
    // map's iteration order then gives the Symbol vector order (:11-14).
    std::unordered_map<int, int> counts;
    for (const auto& sc : first_order_counts) counts.emplace(sc.first, sc.second);
    std::vector<std::pair<int, int>> leaves(counts.begin(), counts.end());
    const int n = (int)leaves.size();

    by_len.assign(17, {});
    if (n == 0) return;
    if (n == 1) {  // Huffman.cpp:17-25
        by_len[1] = {leaves[0].first};
        return;
    }

    // Package nodes: ids [0, n) are leaves, ids >= n are packages (child pair).
    std::vector<std::pair<int, int>> kids;
    kids.reserve((size_t)kLimit * n);

    Level base;
    for (int i = 0; i < n; ++i) base.push(Item{leaves[i].second, i});
    std::vector<Level> levels(kLimit, base);
    levels.emplace_back();
    for (int i = 0; i < kLimit; ++i) {
        Level& lv = levels[i];
        Level& nx = levels[i + 1];
        while (lv.size() > 1) {
            Item a = lv.top(); lv.pop();
            Item b = lv.top(); lv.pop();
            kids.emplace_back(a.node, b.node);
            nx.push(Item{(int)((unsigned)a.weight + (unsigned)b.weight), n + (int)kids.size() - 1});  // (int wrap, as the reference)
        }
    }
    std::vector<int> final_order;
    Level& fin = levels[kLimit];
    while (!fin.empty()) { final_order.push_back(fin.top().node); fin.pop(); }

    // Code length of a symbol = number of times it appears across the final
    // packages (Huffman.hpp:153-161): push multiplicities down the DAG.
    const int total = n + (int)kids.size();
    std::vector<int> mult(total, 0);
    for (int f : final_order) mult[f] += 1;
    for (int id = total - 1; id >= n; --id) {
        if (!mult[id]) continue;
        const auto& k = kids[id - n];
        mult[k.first] += mult[id];
        mult[k.second] += mult[id];
    }

    // Insertion order of code_lengths: final packages in pop order, each one's
    // symbols ascending (std::merge keeps package symbol lists sorted,
    // Huffman.hpp:103-108).  Track each node's distinct-symbol set as a bitset
    // over symbol rank.
    std::vector<int> rank_sym(n);
    std::iota(rank_sym.begin(), rank_sym.end(), 0);
    std::sort(rank_sym.begin(), rank_sym.end(),
              [&](int a, int b) { return leaves[a].first < leaves[b].first; });
    std::vector<int> rank_of(n);
    for (int r = 0; r < n; ++r) rank_of[rank_sym[r]] = r;
    const int words = (n + 63) / 64;
    std::vector<uint64_t> sets((size_t)total * words, 0);
    for (int i = 0; i < n; ++i) sets[(size_t)i * words + rank_of[i] / 64] |= 1ull << (rank_of[i] % 64);
    for (int id = n; id < total; ++id) {
        const auto& k = kids[id - n];
        for (int w = 0; w < words; ++w)
            sets[(size_t)id * words + w] = sets[(size_t)k.first * words + w] | sets[(size_t)k.second * words + w];
    }
    std::vector<char> seen(n, 0);
    std::unordered_map<int, int> code_lengths;
    for (int f : final_order) {
        for (int w = 0; w < words; ++w) {
            uint64_t bits = sets[(size_t)f * words + w];
            while (bits) {
                int r = w * 64 + __builtin_ctzll(bits);
                bits &= bits - 1;
                int leaf = rank_sym[r];
                if (!seen[leaf]) {
                    seen[leaf] = 1;
                    code_lengths.emplace(leaves[leaf].first, mult[leaf]);
                }
            }
        }
    }
    by_len.assign(kLimit + 2, {});
    for (const auto& kv : code_lengths) by_len[kv.second].push_back(kv.first);

    // preventOnlyOnesCode (Huffman.cpp:37-48): move the last symbol of the
    // longest non-empty length one level deeper.
    int last = kLimit + 1;
    while (last > 0 && by_len[last].empty()) --last;
    int s = by_len[last].back();
    by_len[last].pop_back();
    by_len[last + 1].push_back(s);
}

// ---- the same algorithm without standard containers (the per-frame hot path) ----
//
// build_code_lengths_std above feeds std::unordered_map and std::priority_queue; the
// code below reproduces what those containers do, step for step, on fixed arrays:
//  - HashOrder: the iteration order of a libstdc++ std::unordered_map<int, int> after
//    inserting keys in a given order (hash = identity; a new key goes to the front of
//    its bucket, or of the whole list when its bucket is empty; a rehash relinks the
//    list in the same way), with the bucket counts recorded once from a real map;
//  - the binary heap of std::priority_queue<Item, vector<Item>, ItemGreater>: push =
//    std::push_heap, pop = std::pop_heap (libstdc++'s __adjust_heap, then __push_heap),
//    comparing weights only;
//  - packages as a DAG of node ids: a symbol's code length is its number of paths
//    from the final packages (Huffman.hpp:153-161), and code_lengths receives the
//    symbols by (first final package that holds them, symbol), as std::merge keeps a
//    package's symbols sorted (Huffman.hpp:103-108).
// tests/cpp/test_huffman_fast.cpp checks it against build_code_lengths_std and
// std::unordered_map on random inputs; the package-merge golden cases pin both.
namespace {

constexpr int kMaxSyms = 256;

// LSD radix sort of a[0..n) by key(a[i]) (uint64_t, ascending, stable), one counting pass
// per byte that differs among the keys (histogram keys and weights vary in 2-4 bytes).
// Branch-free where std::sort mispredicts about every other comparison on a frame's
// fresh data; n <= 2 * kMaxSyms.
template <class T, class Key>
void radix_sort(T* a, int n, Key key) {
    if (n < 2) return;
    if (n <= 24) {  // (a DC table's ~10 symbols: insertion sort, cheaper than 256-bucket passes)
        for (int i = 1; i < n; ++i) {
            const T v = a[i];
            const uint64_t kv = key(v);
            int j = i - 1;
            while (j >= 0 && key(a[j]) > kv) {
                a[j + 1] = a[j];
                --j;
            }
            a[j + 1] = v;
        }
        return;
    }
    T tmp[2 * kMaxSyms];
    uint64_t diff = 0;
    const uint64_t k0 = key(a[0]);
    for (int i = 1; i < n; ++i) diff |= key(a[i]) ^ k0;
    T* src = a;
    T* dst = tmp;
    for (int sh = 0; sh < 64; sh += 8) {
        if (!((diff >> sh) & 0xFF)) continue;
        uint32_t cnt[257] = {};
        for (int i = 0; i < n; ++i) ++cnt[((key(src[i]) >> sh) & 0xFF) + 1];
        for (int b = 0; b < 256; ++b) cnt[b + 1] += cnt[b];
        for (int i = 0; i < n; ++i) dst[cnt[(key(src[i]) >> sh) & 0xFF]++] = src[i];
        std::swap(src, dst);
    }
    if (src != a) std::copy(src, src + n, a);
}

class HashOrder {
  public:
    // bucket_count() of a std::unordered_map<int, int> after k insertions (k <= kMaxSyms)
    static const uint32_t* buckets() {
        static const std::vector<uint32_t> bc = [] {
            std::vector<uint32_t> v(kMaxSyms + 1);
            std::unordered_map<int, int> m;
            v[0] = (uint32_t)m.bucket_count();
            for (int k = 1; k <= kMaxSyms; ++k) {
                m.emplace(k, k);
                v[k] = (uint32_t)m.bucket_count();
            }
            return v;
        }();
        return bc.data();
    }
    static constexpr uint32_t kMaxBuckets = kMaxSyms + 64;
    // order() sizes its bucket array for libstdc++'s growth policy (at most 257 buckets
    // for 256 keys); a standard library that grows further takes the std-container path
    static bool usable() {
        static const bool ok = [] {
            const uint32_t* bc = buckets();
            for (int k = 0; k <= kMaxSyms; ++k)
                if (bc[k] > kMaxBuckets) return false;
            return true;
        }();
        return ok;
    }
    // key % bucket count for byte keys, per distinct bucket count of buckets() (the
    // modulo was most of order()'s time: a 64-bit division per key and rehash)
    struct ModTable {
        uint32_t nb[kMaxSyms + 1];  // the distinct counts, in growth order
        int cnt = 0;
        uint16_t mod[16][256];
    };
    static const ModTable& mods() {
        static const ModTable t = [] {
            ModTable m;
            const uint32_t* bc = buckets();
            for (int k = 0; k <= kMaxSyms && m.cnt < 16; ++k) {
                if (m.cnt && m.nb[m.cnt - 1] == bc[k]) continue;
                m.nb[m.cnt] = bc[k];
                for (uint32_t x = 0; x < 256; ++x) m.mod[m.cnt][x] = (uint16_t)(x % bc[k]);
                ++m.cnt;
            }
            return m;
        }();
        return t;
    }
    // iteration order (indices into keys) after inserting distinct keys[0..n) (std::hash<int>:
    // the value as size_t, so a negative key hashes to 2^64 + key)
    static void order(const int* keys, int n, int* out) {
        bool bytes = true;
        for (int i = 0; i < n; ++i) bytes &= (uint32_t)keys[i] < 256u;
        const ModTable& mt = mods();
        if (bytes && mt.cnt < 16) order_with(keys, n, out, [&mt](int key, int gen) -> uint32_t {
            return mt.mod[gen][key];
        });
        else order_with(keys, n, out, [&mt](int key, int gen) -> uint32_t {
            return (uint32_t)(static_cast<size_t>(key) % mt.nb[gen]);
        });
    }
    template <class Mod>
    static void order_with(const int* keys, int n, int* out, Mod&& mod) {
        constexpr int kNone = -1, kBefore = -2;  // bucket empty / its predecessor is before_begin
        const uint32_t* bc = buckets();
        int next[kMaxSyms];
        int bucket[kMaxBuckets];  // node before the bucket's first node (usable())
        uint32_t nb = bc[0];
        int gen = 0;  // nb = mods().nb[gen]
        int head = kNone;
        for (uint32_t b = 0; b < nb; ++b) bucket[b] = kNone;
        for (int i = 0; i < n; ++i) {
            if (bc[i + 1] != nb) {  // _M_rehash_aux (unique keys)
                nb = bc[i + 1];
                ++gen;
                for (uint32_t b = 0; b < nb; ++b) bucket[b] = kNone;
                int p = head, bbegin = 0;
                head = kNone;
                while (p != kNone) {
                    const int nx = next[p];
                    const uint32_t b = mod(keys[p], gen);
                    if (bucket[b] == kNone) {
                        next[p] = head;
                        head = p;
                        bucket[b] = kBefore;
                        if (next[p] != kNone) bucket[bbegin] = p;
                        bbegin = (int)b;
                    } else if (bucket[b] == kBefore) {
                        next[p] = head;
                        head = p;
                    } else {
                        next[p] = next[bucket[b]];
                        next[bucket[b]] = p;
                    }
                    p = nx;
                }
            }
            const uint32_t b = mod(keys[i], gen);  // _M_insert_bucket_begin
            if (bucket[b] != kNone) {
                if (bucket[b] == kBefore) {
                    next[i] = head;
                    head = i;
                } else {
                    next[i] = next[bucket[b]];
                    next[bucket[b]] = i;
                }
            } else {
                next[i] = head;
                head = i;
                if (next[i] != kNone) bucket[mod(keys[next[i]], gen)] = i;
                bucket[b] = kBefore;
            }
        }
        int k = 0;
        for (int p = head; p != kNone; p = next[p]) out[k++] = p;
    }
};

// A heap item: weight in the high word, node id in the low word.  Comparisons look at
// the weight only (as the reference's comparator), so equal weights never reorder.  The
// weight is stored with its sign bit flipped, so the high words compare as unsigned
// numbers in the order of the signed weights (item_hi).
using HeapItem = uint64_t;
inline HeapItem item(int w, int node) { return ((uint64_t)((uint32_t)w ^ 0x80000000u) << 32) | (uint32_t)node; }
inline int item_w(HeapItem x) { return (int)((uint32_t)(x >> 32) ^ 0x80000000u); }
inline uint32_t item_hi(HeapItem x) { return (uint32_t)(x >> 32); }
inline int item_node(HeapItem x) { return (int)(uint32_t)x; }
// std::push_heap with comp(a, b) = a.w > b.w (libstdc++ __push_heap)
inline void heap_push(HeapItem* h, int& size, HeapItem v) {
    int hole = size++;
    const int vw = item_w(v);
    while (hole > 0) {
        const int parent = (hole - 1) / 2;
        if (!(item_w(h[parent]) > vw)) break;
        h[hole] = h[parent];
        hole = parent;
    }
    h[hole] = v;
}
// std::pop_heap + pop_back (libstdc++ __pop_heap / __adjust_heap / __push_heap).
// __adjust_heap walks the hole from the root to the bottom, at each node taking the
// right child unless the left one is lighter.  The walk keeps the two children of the
// hole in registers and loads their four children one step ahead, so a step waits on
// a compare, not on a load (the heap arrays carry kHeapPad slack for those loads).
constexpr int kHeapPad = 8;
inline HeapItem heap_pop(HeapItem* h, int& size) {
    const HeapItem top = h[0];
    const int len = size - 1;
    if (len > 0) {
        const HeapItem v = h[len];
        int hole = 0;
        const int lim = (len - 1) / 2;
        if (hole < lim) {
            HeapItem cl = h[1], cr = h[2];
            do {
                const HeapItem* g = h + 4 * hole + 3;  // the children's children (may lie past len)
                const HeapItem g0 = g[0], g1 = g[1], g2 = g[2], g3 = g[3];
                const bool left = item_w(cr) > item_w(cl);
                h[hole] = left ? cl : cr;
                hole = 2 * hole + 2 - (int)left;
                cl = left ? g0 : g2;
                cr = left ? g1 : g3;
            } while (hole < lim);
        }
        if ((len & 1) == 0 && hole == (len - 2) / 2) {
            h[hole] = h[2 * hole + 1];
            hole = 2 * hole + 1;
        }
        const int vw = item_w(v);
        while (hole > 0) {
            const int parent = (hole - 1) / 2;
            if (!(item_w(h[parent]) > vw)) break;
            h[hole] = h[parent];
            hole = parent;
        }
        h[hole] = v;
    }
    size = len;
    return top;
}

// The replays below run this pop on a LIGHT heap: every item heavier than a threshold
// is the marker kHi (heavier than every weight in use).  When only the pops of the light
// items are wanted, their order does not depend on the heavy items' weights:
//  - the hole walks from the root along the lighter child; while a light child exists it
//    is the lighter one, and once both children are heavy (or absent) the rest of the
//    walk moves markers only (equal items: which marker moves is immaterial);
//  - the last item v then enters at the bottom of that walk and rises past every heavier
//    item on it: a heavy v stops below the light items, a light v passes the markers and
//    continues exactly as in the full heap.
// A push is the same: a light item rises past every heavy ancestor and then by weight; a
// heavy one never passes a light item, so it is appended as the marker.  So the light
// items' positions evolve as in the full heap.  (Stopping the walk at the light region's
// edge saves steps but costs a test per step: the full-depth walk is ~1.5% faster.)

// by_len[l] = the symbols of code length l (l = 1..17) in the reference's order;
// syms/cnts: the distinct symbols and counts in first-occurrence order.
void code_lengths_fast(const int* syms, const int* cnts, int n, int by_len[18][kMaxSyms], int nlen[18]) {
    for (int l = 0; l < 18; ++l) nlen[l] = 0;
    if (n <= 0) return;
    // leaves in the iteration order of symbol_counts (Huffman.cpp:6-14)
    int ord[kMaxSyms], lsym[kMaxSyms], lcnt[kMaxSyms];
    HashOrder::order(syms, n, ord);
    for (int i = 0; i < n; ++i) {
        lsym[i] = syms[ord[i]];
        lcnt[i] = cnts[ord[i]];
    }
    if (n == 1) {  // Huffman.cpp:17-25
        by_len[1][nlen[1]++] = lsym[0];
        return;
    }
    // package-merge, Huffman.hpp:114-174: 15 levels, each a copy of the leaves' heap
    // plus the previous level's packages; levels[15] starts empty.
    //
    // A level is filled completely before it is popped (its packages go to the next
    // level), and a binary heap pops in weight order, so a level's pop sequence is its
    // items sorted by weight; the heap decides only the order among EQUAL weights.  The
    // previous level's packages arrive in non-decreasing weight (sums of consecutive
    // pops), so the sorted items are a merge of the sorted leaves and those packages.
    // Consecutive pops pair up into packages, so the order inside a tie matters only
    // when the tie spans more than one pair (or the unpaired last item; on the final
    // level, where every pop counts, any tie).  The heap is therefore run only up to
    // the last such tie of the level; past it the merged order is the pop order (a tie
    // of two inside one pair only swaps a package's two children, which nothing
    // downstream distinguishes).  On 4K frames this leaves 0-11% of the reference's
    // heap pops to simulate.
    constexpr int kLevels = 15, kCap = 2 * kMaxSyms;
    constexpr int kMaxKids = kLevels * kCap, kMaxNodes = kMaxSyms + kMaxKids;
    // (the heap is padded for heap_pop's look-ahead loads; the lists that are merged
    // carry a sentinel slot at each end: index -1 and index size)
    // A per-thread workspace, reached through a pointer loaded once: in a shared library
    // every access to a thread_local array is a __tls_get_addr call, and the compiler
    // recomputes such addresses inside loops instead of keeping them (4 tables of a
    // 1080p frame took 56 us in the library against 20 us linked statically).
    struct Work {
        HeapItem base[kMaxSyms], heap[2 * kCap + kHeapPad], srt_[2 * kCap + 3];
        HeapItem rp_pop[2 * kCap];
        uint32_t rp_w[kCap];
        HeapItem pk_[2][kCap + 2], lsrt_[kMaxSyms + 2];
        int kid_a[kMaxKids], kid_b[kMaxKids], mult[kMaxNodes], first[kMaxNodes];
    };
    static thread_local std::unique_ptr<Work> tls_work;
    Work* wp = tls_work.get();
    if (!wp) {
        tls_work.reset(new Work());
        wp = tls_work.get();
    }
    Work& W = *wp;
    HeapItem* const base = W.base;
    HeapItem* const heap = W.heap;
    HeapItem* const srt_ = W.srt_;
    HeapItem(*const pk_)[kCap + 2] = W.pk_;
    HeapItem* const lsrt_ = W.lsrt_;
    constexpr HeapItem kLo = 0, kHi = ~0ull;  // sentinels: below / above every weight in use
    int nbase = 0;
    for (int i = 0; i < n; ++i) heap_push(base, nbase, item(lcnt[i], i));
    HeapItem* const lsrt = lsrt_ + 1;  // the leaves by weight
    HeapItem* const srt = srt_ + 1;    // a level's pop order
    for (int i = 0; i < n; ++i) lsrt[i] = item(lcnt[i], i);
    radix_sort(lsrt, n, [](HeapItem x) -> uint64_t { return item_hi(x); });
    lsrt[-1] = pk_[0][0] = kLo;
    lsrt[n] = pk_[0][1] = kHi;  // (levels[0]: no packages)
    int* const kid_a = W.kid_a;
    int* const kid_b = W.kid_b;
    int* const mult = W.mult;
    int* const first = W.first;
    int nkids = 0, np = 0;
    struct LightReplay {  // the last light replay's inputs and pops
        bool valid = false;
        uint32_t wl = 0, pbase = 0;
        int e = -1, np = 0, nl = 0;
        uint32_t* w;
        HeapItem* pop;
    } rp;
    rp.w = W.rp_w;
    rp.pop = W.rp_pop;
    // Weights are the reference's ints.  The merges need every weight strictly between the
    // sentinels; if a package's sum reaches 2^31 - 1 or wraps (counts near 2^31), the
    // later levels run the heap whole instead.
    bool wrapped = false;
    for (int i = 0; i < n; ++i) wrapped |= lcnt[i] <= INT32_MIN + 1 || lcnt[i] >= INT32_MAX;
    // The end (inclusive) of the last tie in srt[0, m) whose order the heap decides, -1 if
    // none.  eq[k]: item k weighs the same as item k-1.  A tie between k-1 and k is
    // harmless only when they are one pair (k odd, below pe = the paired items) and the
    // tie reaches neither k-2 nor k+1; a harmful tie's later items are harmful too, so
    // the last harmful k is the end of the last harmful tie.  (Branch-free.)
    // (the flags of k-1, k and k+1 ride in registers; srt[m] = kHi ends the last tie)
    auto last_tie = [srt](int m, int pe) {
        srt[m] = kHi;
        int e = -1;
        uint32_t hc = item_hi(srt[0]), hn = item_hi(srt[1]);
        bool ep = false, ec = hn == hc;  // eq[k-1], eq[k] for k = 1
        hc = hn;
        for (int k = 1; k < m; ++k) {
            hn = item_hi(srt[k + 1]);
            const bool en = hn == hc;  // eq[k+1]
            const bool h = ec & (((k & 1) == 0) | ep | en | (k >= pe));
            e = h ? k : e;
            ep = ec;
            ec = en;
            hc = hn;
        }
        return e;
    };
    // One level, merged: levels[lv] = the leaves + levels[lv-1]'s packages by weight,
    // leaves first on ties, as two branch-free chains run from both ends at once (a chain
    // step waits on its loads, so two in flight halve the wait).  The chains also pair
    // consecutive items into this level's packages and mark ties (eq bit k: item k
    // weighs as item k-1), which then give the last tie the heap decides (last_tie's rule
    // on 64 positions at a time).  A heap replay up to that tie changes only which equal
    // weights stand where, so the packages' weights stay and only their children are
    // taken again.
    constexpr int kEqWords = (2 * kCap + 64) / 64 + 1;
    constexpr uint64_t kEven = 0x5555555555555555ull;  // (bit k: k even)
    auto merge_level = [&](const HeapItem* in, HeapItem* out, int m, int npairs, bool& wrap) {
        const int half = (m + 1) / 2, nk = nkids;
        uint64_t E[kEqWords];
        const int words = (m >> 6) + 1;  // (positions 0..m)
        for (int w = 0; w < words; ++w) E[w] = 0;
        int i = 0, j = 0, i2 = n - 1, j2 = np - 1;
        HeapItem pf = kLo, pb = kHi;  // the front chain's previous item (k - 1), the back chain's (p + 1)
        uint64_t accf = 0, accb = 0;
        bool wr = false;
        auto pair = [&](int q, HeapItem a, HeapItem b) {
            kid_a[nk + q] = item_node(a);
            kid_b[nk + q] = item_node(b);
            const int64_t sum = (int64_t)item_w(a) + item_w(b);
            wr |= sum >= INT32_MAX || sum <= INT32_MIN + 1;
            out[q] = item((int32_t)(uint32_t)sum, n + nk + q);
        };
        for (int k = 0; k < half; ++k) {
            const int p = m - 1 - k;
            // from the end (an odd m's middle item is written by both chains)
            const HeapItem a2 = lsrt[i2], b2 = in[j2];
            const bool t2 = item_hi(b2) >= item_hi(a2);
            const HeapItem cb = t2 ? b2 : a2;
            srt[p] = cb;
            j2 -= t2;
            i2 -= !t2;
            accb |= (uint64_t)(item_hi(pb) == item_hi(cb)) << ((p + 1) & 63);  // eq[p + 1]
            if (((p + 1) & 63) == 0) {
                E[(p + 1) >> 6] |= accb;
                accb = 0;
            }
            if (!(p & 1) && (p >> 1) < npairs) pair(p >> 1, cb, pb);
            pb = cb;
            // from the front
            const HeapItem a = lsrt[i], b = in[j];
            const bool t = item_hi(b) < item_hi(a);
            const HeapItem cf = t ? b : a;
            srt[k] = cf;
            j += t;
            i += !t;
            accf |= (uint64_t)(item_hi(cf) == item_hi(pf)) << (k & 63);  // eq[k]
            if ((k & 63) == 63) {
                E[k >> 6] |= accf;
                accf = 0;
            }
            if (k & 1) pair(k >> 1, pf, cf);
            pf = cf;
        }
        E[(half - 1) >> 6] |= accf;
        E[(m - half + 1) >> 6] |= accb;
        if (!(m & 1) && m >= 2) {  // (the middle tie of an even m: between the chains)
            const int c = m / 2;
            E[c >> 6] |= (uint64_t)(item_hi(srt[c]) == item_hi(srt[c - 1])) << (c & 63);
        }
        for (int q = half >> 1; q < ((m - half + 1) >> 1) && q < npairs; ++q) pair(q, srt[2 * q], srt[2 * q + 1]);
        srt[-1] = kLo;
        srt[m] = kHi;
        wrap |= wr;
        // the last harmful tie: eq[k] and (k even, eq[k-1], eq[k+1] or k past the pairs)
        const int pe = m - (m & 1);
        for (int w = words - 1; w >= 0; --w) {
            const uint64_t prv = (E[w] << 1) | (w ? E[w - 1] >> 63 : 0ull);
            const uint64_t nxt = (E[w] >> 1) | (w + 1 < words ? E[w + 1] << 63 : 0ull);
            const int b0 = 64 * w;
            const uint64_t ge = pe <= b0 ? ~0ull : pe >= b0 + 64 ? 0ull : ~0ull << (pe - b0);
            const uint64_t H = E[w] & (kEven | prv | nxt | ge);
            if (H) return b0 + 63 - __builtin_clzll(H);
        }
        return -1;
    };
    int prev_np = -1;  // the previous level's package count (its input)
    for (int lv = 0; lv < kLevels; ++lv) {
        const HeapItem* in = pk_[lv & 1] + 1;
        HeapItem* out = pk_[(lv + 1) & 1] + 1;
        const int m = n + np, npairs = m / 2;
        bool wrap_next = false;
        // A level whose packages weigh exactly what the previous level's did (the levels
        // converge: ~21% of a 1080p frame's) is that level again: the same merge, ties and
        // replay, so the same pairs of positions; only the package ids differ, by the
        // distance between the two levels' package numbers.  Its packages then weigh what
        // its input does.  (The previous level's input is this level's output buffer.)
        if (!wrapped && np > 0 && np == prev_np && npairs == np) {
            bool same = true;
            for (int k = 0; k < np; ++k) same &= item_hi(in[k]) == item_hi(out[k]);
            if (same) {
                const uint32_t shift = (uint32_t)item_node(in[0]) - (uint32_t)item_node(out[0]);
                for (int q = 0; q < npairs; ++q) {
                    const int a = kid_a[nkids - np + q], b = kid_b[nkids - np + q];
                    kid_a[nkids + q] = a >= n ? (int)((uint32_t)a + shift) : a;
                    kid_b[nkids + q] = b >= n ? (int)((uint32_t)b + shift) : b;
                    out[q] = (in[q] & 0xFFFFFFFF00000000ull) | (uint32_t)(n + nkids + q);
                }
                nkids += npairs;
                out[-1] = kLo;
                out[npairs] = kHi;
                prev_np = np;
                np = npairs;
                continue;
            }
        }
        prev_np = np;
        if (wrapped) {  // the reference's heap: the leaves' heap, then the pushes, every pop
            const int e = 2 * npairs - 1;
            int hn = nbase;
            std::copy(base, base + nbase, heap);
            for (int k = 0; k < np; ++k) heap_push(heap, hn, in[k]);
            for (int k = 0; k <= e; ++k) srt[k] = heap_pop(heap, hn);
            for (int k = 0; k < npairs; ++k) {
                const HeapItem a = srt[2 * k], b = srt[2 * k + 1];
                kid_a[nkids + k] = item_node(a);
                kid_b[nkids + k] = item_node(b);
                out[k] = item((int32_t)((uint32_t)item_w(a) + (uint32_t)item_w(b)), n + nkids + k);
            }
        } else {
            const int e = merge_level(in, out, m, npairs, wrap_next);
            if (e >= 0) {  // the heap up to that tie, on its light items (a light heap)
                const uint32_t wl = item_hi(srt[e]);  // (the tie ends at e: exactly srt[0..e] are light)
                int nl = 0;  // the light packages (they come in weight order)
                while (nl < np && item_hi(in[nl]) <= wl) ++nl;
                // The light replay depends only on the threshold, the light packages'
                // weights and the heap's size (the leaves are the same every level, the
                // heavy items markers): when those equal the previous replay's, so do the
                // pops, slot for slot, with each package replaced by its counterpart of
                // this level (on 1080p frames the light items repeat on about half the
                // levels).
                bool same = rp.valid && wl == rp.wl && e == rp.e && np == rp.np && nl == rp.nl;
                for (int k = 0; same && k < nl; ++k) same = item_hi(in[k]) == rp.w[k];
                const uint32_t pbase = np ? (uint32_t)item_node(in[0]) : 0u;  // (packages are numbered in order)
                if (same) {
                    const uint32_t shift = pbase - rp.pbase;
                    for (int k = 0; k <= e; ++k) {
                        const HeapItem x = rp.pop[k];
                        srt[k] = x + ((uint32_t)item_node(x) >= (uint32_t)n ? (HeapItem)shift : 0);
                    }
                } else {
                    for (int k = 0; k < nbase; ++k) heap[k] = item_hi(base[k]) > wl ? kHi : base[k];
                    int hn = nbase;
                    for (int k = 0; k < nl; ++k) heap_push(heap, hn, in[k]);
                    std::fill(heap + hn, heap + nbase + np, kHi);
                    hn = nbase + np;
                    for (int k = 0; k <= e; ++k) srt[k] = heap_pop(heap, hn);
                    rp.valid = true;
                    rp.wl = wl;
                    rp.e = e;
                    rp.np = np;
                    rp.nl = nl;
                    for (int k = 0; k < nl; ++k) rp.w[k] = item_hi(in[k]);
                }
                std::copy(srt, srt + e + 1, rp.pop);
                rp.pbase = pbase;
                for (int q = 0; q <= (e >> 1) && q < npairs; ++q) {  // (the replayed pairs' children)
                    kid_a[nkids + q] = item_node(srt[2 * q]);
                    kid_b[nkids + q] = item_node(srt[2 * q + 1]);
                }
            }
        }
        nkids += npairs;
        wrapped |= wrap_next;
        out[-1] = kLo;
        out[npairs] = kHi;
        np = npairs;
    }
    // levels[15]: levels[14]'s packages alone, pushed in non-decreasing weight, so its
    // heap array is the push order; its pop order = the final packages.  (Every pop
    // counts here, so every tie is the heap's.)
    const HeapItem* fin = pk_[kLevels & 1] + 1;
    std::copy(fin, fin + np, srt);
    srt[-1] = kLo;
    const int e = wrapped ? np - 1 : last_tie(np, 0);
    if (e >= 0 && wrapped) {
        int hn = 0;
        for (int k = 0; k < np; ++k) heap_push(heap, hn, fin[k]);
        for (int k = 0; k <= e; ++k) srt[k] = heap_pop(heap, hn);
    } else if (e >= 0) {
        const uint32_t wl = item_hi(srt[e]);
        for (int k = 0; k < np; ++k) heap[k] = item_hi(fin[k]) > wl ? kHi : fin[k];
        int hn = np;
        for (int k = 0; k <= e; ++k) srt[k] = heap_pop(heap, hn);
    }
    // Push the multiplicities and the first final package down the DAG (a package's id
    // exceeds its children's).
    const int total = n + nkids;
    std::fill(mult, mult + total, 0);
    std::fill(first, first + total, INT32_MAX);
    for (int k = 0; k < np; ++k) {
        const int f = item_node(srt[k]);
        mult[f] += 1;
        if (k < first[f]) first[f] = k;
    }
    for (int id = total - 1; id >= n; --id) {  // (unused packages add 0: no branch)
        const int ka = kid_a[id - n], kb = kid_b[id - n];
        mult[ka] += mult[id];
        mult[kb] += mult[id];
        first[ka] = std::min(first[ka], first[id]);
        first[kb] = std::min(first[kb], first[id]);
    }
    // code_lengths (an unordered_map) receives symbols by (first package, symbol)
    int ins[kMaxSyms];
    for (int i = 0; i < n; ++i) ins[i] = i;
    radix_sort(ins, n, [&](int x) -> uint64_t {
        return ((uint64_t)(uint32_t)first[x] << 32) | ((uint32_t)lsym[x] ^ 0x80000000u);  // (signed symbols)
    });
    int ksym[kMaxSyms];
    for (int i = 0; i < n; ++i) ksym[i] = lsym[ins[i]];
    HashOrder::order(ksym, n, ord);
    for (int i = 0; i < n; ++i) {
        const int leaf = ins[ord[i]], l = mult[leaf];
        by_len[l][nlen[l]++] = lsym[leaf];
    }
    // preventOnlyOnesCode (Huffman.cpp:37-48): the last symbol of the longest length
    // moves one level deeper
    int last = 16;
    while (last > 0 && nlen[last] == 0) --last;
    const int sv = by_len[last][--nlen[last]];
    by_len[last + 1][nlen[last + 1]++] = sv;
}

}  // namespace

void build_code_lengths(const std::vector<std::pair<int, int>>& first_order_counts,
                        std::vector<std::vector<int>>& by_len) {
    const int n = (int)first_order_counts.size();
    if (n > kMaxSyms || !HashOrder::usable()) {  // (symbol texts beyond byte symbols: the facade only)
        build_code_lengths_std(first_order_counts, by_len);
        return;
    }
    by_len.assign(17, {});
    if (n == 0) return;
    int syms[kMaxSyms], cnts[kMaxSyms];
    for (int i = 0; i < n; ++i) {
        syms[i] = first_order_counts[i].first;
        cnts[i] = first_order_counts[i].second;
    }
    static thread_local int bl[18][kMaxSyms];
    int nl[18];
    code_lengths_fast(syms, cnts, n, bl, nl);
    by_len.assign(17, {});  // (lengths <= 16: package-merge limits them to 15, +1 for preventOnlyOnesCode)
    for (int l = 0; l < 17; ++l) by_len[l].assign(bl[l], bl[l] + nl[l]);
}

std::vector<std::pair<int, GenericCode>> assign_codes(const std::vector<std::vector<int>>& by_len) {
    // generateCodes (Huffman.cpp:50-66): canonical codes in SymbolsPerLength order.
    std::vector<std::pair<int, GenericCode>> out;
    uint32_t c = 0;
    for (int l = 1; l < (int)by_len.size(); ++l) {
        for (int s : by_len[l]) out.push_back({s, GenericCode{c++, l}});
        c <<= 1;
    }
    return out;
}

static bool build_table_with(const uint32_t counts[256], const uint64_t first_key[256], HuffTable& out,
                             void (*lengths)(const std::vector<std::pair<int, int>>&, std::vector<std::vector<int>>&)) {
    std::vector<std::pair<uint64_t, int>> order;
    for (int s = 0; s < 256; ++s)
        if (counts[s]) order.emplace_back(first_key[s], s);
    if (order.empty()) return false;
    std::sort(order.begin(), order.end());
    std::vector<std::pair<int, int>> fc;
    fc.reserve(order.size());
    for (const auto& o : order) fc.emplace_back(o.second, (int)counts[o.second]);

    std::vector<std::vector<int>> by_len;
    lengths(fc, by_len);
    out = HuffTable();
    int k = 0;
    for (int l = 1; l <= 16 && l < (int)by_len.size(); ++l) {
        out.bits[l] = (uint8_t)by_len[l].size();
        for (int s : by_len[l]) out.huffval[k++] = (uint8_t)s;
    }
    out.nsym = k;
    for (const auto& sc : assign_codes(by_len)) {
        out.code[sc.first & 0xFF] = sc.second.code;
        out.len[sc.first & 0xFF] = (uint8_t)sc.second.length;
    }
    return true;
}

bool build_table_std(const uint32_t counts[256], const uint64_t first_key[256], HuffTable& out) {
    return build_table_with(counts, first_key, out, build_code_lengths_std);
}

// kInv: the keys arrive inverted (~first occurrence: the device's atomicMax form, read
// straight from the mapped histogram export)
template <bool kInv>
static bool build_table_impl(const uint32_t counts[256], const uint64_t keys[256], HuffTable& out) {
    // symbols in first-occurrence order
    uint64_t key[kMaxSyms];
    int syms[kMaxSyms], cnts[kMaxSyms], n = 0;
    for (int s = 0; s < 256; ++s)
        if (counts[s]) {
            key[n] = ((kInv ? ~keys[s] : keys[s]) << 8) | (uint64_t)s;  // (keys are < 2^56: text positions)
            ++n;
        }
    if (!n) return false;
    radix_sort(key, n, [](uint64_t k) { return k; });
    for (int i = 0; i < n; ++i) {
        syms[i] = (int)(key[i] & 0xFF);
        cnts[i] = (int)counts[syms[i]];
    }
    int bl[18][kMaxSyms], nl[18];
    code_lengths_fast(syms, cnts, n, bl, nl);
    out = HuffTable();
    // canonical codes in SymbolsPerLength order (generateCodes, Huffman.cpp:50-66)
    int k = 0;
    uint32_t c = 0;
    for (int l = 1; l < 18; ++l) {
        if (l <= 16) out.bits[l] = (uint8_t)nl[l];
        for (int i = 0; i < nl[l]; ++i) {
            const int sv = bl[l][i];
            if (l <= 16) out.huffval[k++] = (uint8_t)sv;
            out.code[sv & 0xFF] = c++;
            out.len[sv & 0xFF] = (uint8_t)l;
        }
        c <<= 1;
    }
    out.nsym = k;
    return true;
}

bool build_table(const uint32_t counts[256], const uint64_t first_key[256], HuffTable& out) {
    if (!HashOrder::usable()) return build_table_std(counts, first_key, out);
    return build_table_impl<false>(counts, first_key, out);
}

bool build_table_inverted(const uint32_t counts[256], const uint64_t inv_key[256], HuffTable& out) {
    if (!HashOrder::usable()) {
        uint64_t first[256];
        for (int s = 0; s < 256; ++s) first[s] = ~inv_key[s];
        return build_table_std(counts, first, out);
    }
    return build_table_impl<true>(counts, inv_key, out);
}

std::pair<std::vector<std::pair<int, GenericCode>>, std::vector<std::vector<int>>>
generateHuffmanCode(const std::vector<int>& text) {
    std::unordered_map<int, size_t> index;
    std::vector<std::pair<int, int>> fc;
    for (int s : text) {
        auto it = index.find(s);
        if (it == index.end()) { index.emplace(s, fc.size()); fc.emplace_back(s, 1); }
        else fc[it->second].second++;
    }
    std::vector<std::vector<int>> by_len;
    build_code_lengths(fc, by_len);
    return {assign_codes(by_len), by_len};
}

}  // namespace jpge
