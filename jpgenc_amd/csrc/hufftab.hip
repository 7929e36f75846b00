// Huffman tables on the device (gfx950): generateHuffmanCode (Huffman.cpp:3-66) with
// package_merge (Huffman.hpp:114-174) on libstdc++'s unordered_map and
// priority_queue, for the four tables of a frame, from K2's histograms and
// first-occurrence keys.  The output equals huffman.cpp's build_table bit for bit:
// the per-symbol codes (len << 16 | code) and each table's DHT piece.
//
// The reference's steps and how they run here, one workgroup per table:
//  1. symbol_counts, an unordered_map<int,int> filled in text order: its iteration
//     order after the k-th insertion.  libstdc++ keeps one list: a key entering an
//     empty bucket goes to the list's head, any other to the front of its bucket's
//     run, and a rehash re-inserts the list in order by the same rule.  So between
//     two rehashes the list is the buckets in reverse order of first arrival, each
//     bucket's keys in reverse arrival; the arrivals of an epoch are the previous
//     epoch's list, then the new keys.  Bucket counts after k insertions (1, 13, 29,
//     59, 127, 257) are libstdc++'s; each epoch is one lane-parallel ranking.
//  2. package_merge: 15 levels, each a priority_queue that starts as the leaves
//     (pushed in map order) and receives the previous level's packages in the order
//     they were made.  A heap pops in weight order, so the packages' WEIGHTS at every
//     level follow from a weight-only pass (sorted merges); with them each level's
//     heap is simulated alone: 15 levels and the final level on 16 lanes at once,
//     every push and pop as libstdc++'s __push_heap / __adjust_heap move items,
//     comparing weights only.  The pops give each level's pairs (the packages'
//     children).
//  3. code lengths: each final package counts once for each symbol in it; the counts
//     go down the package DAG level by level (lane-parallel), with the first final
//     package holding each symbol (code_lengths' insertion order: by that package,
//     then by symbol, as std::merge keeps a package's symbols sorted).
//  4. code_lengths is an unordered_map too: its iteration order (step 1's rule)
//     orders the symbols of each length; preventOnlyOnesCode moves the last symbol
//     of the longest length one deeper; generateCodes numbers them canonically.
// tests/test_gpu_hufftab.py compares every table with the host builder (pinned to
// the reference's own Huffman.cpp) on the golden cases and thousands of random and
// tie-heavy histograms.
#include "device_common.hpp"

namespace jpge {
namespace {
using namespace dev;

constexpr int kTThreads = 256;
constexpr int kLevels = 15;                 // package_merge(symbols, 15)
constexpr int kHeapCap = 2 * 256 + 8;       // a level's items, at most (+ slack for the look-ahead loads)

struct TabLds {
    uint64_t heap[kLevels + 1][kHeapCap];   // per level: items (weight << 32 | node id); [15]: the final level
    uint32_t pkw[kLevels][256];             // weights of the packages level lv makes, in order
    uint32_t pair[kLevels][256];            // their children: node id a << 16 | b
    uint32_t mult[(kLevels + 1) * 256];     // per node id: final packages holding it (code length for a leaf)
    uint32_t firstp[(kLevels + 1) * 256];   // per node id: the first final package holding it
    uint32_t cnt[256];
    uint64_t fk[256];                       // first-occurrence key per symbol (present ones)
    uint32_t order[256], order2[256];       // symbol lists: first-occurrence order / map order work
    uint32_t arr[256];                      // an epoch's arrivals
    uint32_t fv[256];                       // per arrival: its bucket's first arrival
    uint32_t fa[264];                       // first arrival per bucket
    uint32_t leafsym[256], leafw[256], sl[256];
    uint32_t items[512];                    // a level's sorted weights
    uint32_t finalord[256];                 // final level pops: package ids
    uint32_t len[256];                      // per leaf: code length
    uint32_t np[kLevels + 1];               // packages made by each level
    uint32_t bits[18];
    uint32_t n;
};

// node ids: leaf i (map order) = i; package j made by level lv = 256 * (lv + 1) + j
__device__ __forceinline__ uint32_t pkg_id(uint32_t lv, uint32_t j) { return 256u * (lv + 1) + j; }
__device__ __forceinline__ uint32_t item_w(uint64_t x) { return (uint32_t)(x >> 32); }

// std::push_heap with comp(a, b) = a.w > b.w (libstdc++ __push_heap), on one lane's heap
__device__ void heap_push(uint64_t* h, uint32_t& size, uint64_t v) {
    uint32_t hole = size++;
    const uint32_t vw = item_w(v);
    while (hole > 0) {
        const uint32_t parent = (hole - 1) / 2;
        const uint64_t p = h[parent];
        if (!(item_w(p) > vw)) break;
        h[hole] = p;
        hole = parent;
    }
    h[hole] = v;
}
// std::pop_heap + pop_back (libstdc++ __pop_heap / __adjust_heap / __push_heap)
__device__ uint64_t heap_pop(uint64_t* h, uint32_t& size) {
    const uint64_t top = h[0];
    const uint32_t len = size - 1;
    if (len > 0) {
        const uint64_t v = h[len];
        uint32_t hole = 0;
        const uint32_t lim = (len - 1) / 2;
        if (hole < lim) {
            uint64_t cl = h[1], cr = h[2];
            do {  // the hole walks down: the right child unless the left one is lighter
                const uint64_t* g = h + 4 * hole + 3;  // (grandchildren, loaded a step ahead; may lie past len)
                const uint64_t g0 = g[0], g1 = g[1], g2 = g[2], g3 = g[3];
                const bool left = item_w(cr) > item_w(cl);
                h[hole] = left ? cl : cr;
                hole = 2 * hole + 2 - (left ? 1u : 0u);
                cl = left ? g0 : g2;
                cr = left ? g1 : g3;
            } while (hole < lim);
        }
        if ((len & 1) == 0 && hole == (len - 2) / 2) {
            h[hole] = h[2 * hole + 1];
            hole = 2 * hole + 1;
        }
        const uint32_t vw = item_w(v);
        while (hole > 0) {
            const uint32_t parent = (hole - 1) / 2;
            const uint64_t p = h[parent];
            if (!(item_w(p) > vw)) break;
            h[hole] = p;
            hole = parent;
        }
        h[hole] = v;
    }
    size = len;
    return top;
}

// libstdc++ unordered_map<int, int>::bucket_count() after k insertions
__device__ __forceinline__ uint32_t buckets_after(uint32_t k) {
    return k == 0 ? 1u : k <= 13 ? 13u : k <= 29 ? 29u : k <= 59 ? 59u : k <= 127 ? 127u : 257u;
}

// Iteration order of an unordered_map<int, int> after inserting n distinct keys,
// ikey[r] being the r-th inserted: out[m] = the insertion rank of the m-th entry
// iterated.  Uses L.arr and L.fa; all threads call it.
__device__ void map_order(TabLds& L, const uint32_t* ikey, uint32_t n, uint32_t* out, int tid) {
    uint32_t m = 0;  // entries in the list so far (out[0..m))
    while (m < n) {
        // an epoch: the rehash before insertion m (to buckets_after(m + 1) buckets), then
        // the insertions up to the next rehash
        const uint32_t end = m < 13 ? min(n, 13u) : m < 29 ? min(n, 29u) : m < 59 ? min(n, 59u)
                                                                 : m < 127 ? min(n, 127u) : n;
        const uint32_t nb = buckets_after(m + 1);
        for (uint32_t x = tid; x < end; x += kTThreads) L.arr[x] = x < m ? out[x] : x;  // arrivals
        for (uint32_t b = tid; b < nb; b += kTThreads) L.fa[b] = 0xFFFFFFFFu;
        __syncthreads();
        for (uint32_t x = tid; x < end; x += kTThreads) atomicMin(&L.fa[ikey[L.arr[x]] % nb], x);
        __syncthreads();
        for (uint32_t x = tid; x < end; x += kTThreads) L.fv[x] = L.fa[ikey[L.arr[x]] % nb];
        __syncthreads();
        // an entry's place: the entries of buckets first reached later, then the later
        // arrivals of its own bucket
        for (uint32_t x = tid; x < end; x += kTThreads) {
            const uint32_t f = L.fv[x];
            uint32_t pos = 0;
            for (uint32_t y = 0; y < end; ++y) {
                const uint32_t fy = L.fv[y];
                pos += (fy > f || (fy == f && y > x)) ? 1u : 0u;
            }
            out[pos] = L.arr[x];
        }
        __syncthreads();
        m = end;
    }
}

__global__ __launch_bounds__(kTThreads) void huff_tables_kernel(TabArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    TabLds& L = *reinterpret_cast<TabLds*>(smem);
    const int tid = threadIdx.x;
    const uint32_t t = blockIdx.x, set = blockIdx.y;  // table (0 Y-DC, 1 Y-AC, 2 C-DC, 3 C-AC), histogram set
    const uint32_t* cnt = a.cnt + (uint64_t)set * a.cnt_stride + t * 256;
    const uint64_t* key = a.key + (uint64_t)set * a.key_stride + t * 256;
    uint32_t* tab = a.tab + (uint64_t)set * a.tab_stride + t * 256;
    uint8_t* dht = a.dht + (uint64_t)set * a.dht_stride + t * kDhtPiece;
    uint32_t* nsym = a.nsym + (uint64_t)set * a.nsym_stride + t;
    uint64_t* dbg = a.dbg ? a.dbg + ((uint64_t)set * 4 + t) * 16 : nullptr;
#define TSTAMP(i) do { if (dbg && tid == 0) dbg[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
    TSTAMP(0);

    // ---- the symbols in first-occurrence order (Huffman.cpp:6-14 fills the map in text order) ----
    for (uint32_t s = tid; s < 256; s += kTThreads) {
        uint32_t c = 0;
        for (uint32_t r = 0; r < a.replicas; ++r) c += cnt[(uint64_t)r * 1024 + s];
        L.cnt[s] = c;
        L.fk[s] = ~key[s];
        tab[s] = 0;
    }
    if (tid == 0) L.n = 0;
    __syncthreads();
    for (uint32_t s = tid; s < 256; s += kTThreads) {
        if (!L.cnt[s]) continue;
        atomicAdd(&L.n, 1u);
        const uint64_t k = L.fk[s];
        uint32_t r = 0;
        for (uint32_t x = 0; x < 256; ++x) r += (L.cnt[x] && (L.fk[x] < k || (L.fk[x] == k && x < s))) ? 1u : 0u;
        L.order[r] = s;
    }
    __syncthreads();
    const uint32_t n = L.n;
    if (n == 0) {  // (no symbols: no table; a frame always has them, the caller checks)
        if (tid == 0) *nsym = 0;
        return;
    }
    if (n == 1) {  // Huffman.cpp:17-25: the single symbol gets the code 0 of length 1
        if (tid == 0) {
            const uint32_t s = L.order[0];
            tab[s] = 1u << 16;
            dht[0] = (uint8_t)(((t & 1) << 4) | (t >> 1));
            for (int l = 1; l <= 16; ++l) dht[l] = l == 1 ? 1 : 0;
            dht[17] = (uint8_t)s;
            *nsym = 1;
        }
        return;
    }

    TSTAMP(1);
    // ---- 1. leaves in symbol_counts' iteration order (the blueprint's push order) ----
    map_order(L, L.order, n, L.order2, tid);
    for (uint32_t i = tid; i < n; i += kTThreads) {
        const uint32_t s = L.order[L.order2[i]];
        L.leafsym[i] = s;
        L.leafw[i] = L.cnt[s];
    }
    __syncthreads();

    TSTAMP(2);
    // ---- 2a. weight-only pass: each level's package weights (its items popped in order) ----
    // sorted leaf weights
    for (uint32_t i = tid; i < n; i += kTThreads) {
        const uint32_t w = L.leafw[i];
        uint32_t r = 0;
        for (uint32_t x = 0; x < n; ++x) r += (L.leafw[x] < w || (L.leafw[x] == w && x < i)) ? 1u : 0u;
        L.sl[r] = w;
    }
    __syncthreads();
    uint32_t p = 0;  // packages of the previous level
    for (uint32_t lv = 0; lv < (uint32_t)kLevels; ++lv) {
        const uint32_t* prev = lv ? L.pkw[lv - 1] : nullptr;
        // merge the sorted leaves and the previous level's (sorted) packages
        for (uint32_t i = tid; i < n; i += kTThreads) {
            const uint32_t w = L.sl[i];
            uint32_t r = i;
            for (uint32_t x = 0; x < p; ++x) r += prev[x] < w ? 1u : 0u;
            L.items[r] = w;
        }
        for (uint32_t j = tid; j < p; j += kTThreads) {
            const uint32_t w = prev[j];
            uint32_t r = j;
            for (uint32_t x = 0; x < n; ++x) r += L.sl[x] <= w ? 1u : 0u;
            L.items[r] = w;
        }
        __syncthreads();
        const uint32_t np = (n + p) / 2;
        for (uint32_t j = tid; j < np; j += kTThreads) L.pkw[lv][j] = L.items[2 * j] + L.items[2 * j + 1];
        if (tid == 0) L.np[lv] = np;
        __syncthreads();
        p = np;
    }

    TSTAMP(3);
    // ---- 2b. the blueprint heap (leaves pushed in map order), copied to every level ----
    if (tid == 0) {
        uint32_t sz = 0;
        for (uint32_t i = 0; i < n; ++i) heap_push(L.heap[0], sz, ((uint64_t)L.leafw[i] << 32) | i);
    }
    __syncthreads();
    for (uint32_t x = tid; x < (uint32_t)(kLevels - 1) * n; x += kTThreads) L.heap[1 + x / n][x % n] = L.heap[0][x % n];
    for (uint32_t x = tid; x < (uint32_t)(kLevels + 1) * 256; x += kTThreads) {
        L.mult[x] = 0;
        L.firstp[x] = 0xFFFFFFFFu;
    }
    __syncthreads();

    TSTAMP(4);
    // ---- 2c. the 15 levels and the final level, one lane each ----
    if (tid < kLevels + 1) {
        const uint32_t lv = (uint32_t)tid;
        uint64_t* h = L.heap[lv];
        uint32_t sz = lv < (uint32_t)kLevels ? n : 0;
        if (lv > 0) {  // the previous level's packages, in the order it made them
            const uint32_t pp = L.np[lv - 1];
            for (uint32_t j = 0; j < pp; ++j) heap_push(h, sz, ((uint64_t)L.pkw[lv - 1][j] << 32) | pkg_id(lv - 1, j));
        }
        if (lv < (uint32_t)kLevels) {
            for (uint32_t j = 0; sz > 1; ++j) {  // package the two lightest while there are two
                const uint64_t x = heap_pop(h, sz), y = heap_pop(h, sz);
                L.pair[lv][j] = ((uint32_t)x << 16) | ((uint32_t)y & 0xFFFFu);
            }
        } else {
            for (uint32_t k = 0; sz > 0; ++k) L.finalord[k] = (uint32_t)heap_pop(h, sz);
        }
    }
    __syncthreads();

    TSTAMP(5);
    // ---- 3. code lengths down the package DAG (Huffman.hpp:153-161) ----
    {
        const uint32_t nf = L.np[kLevels - 1];
        for (uint32_t k = tid; k < nf; k += kTThreads) {  // every final package once
            const uint32_t id = L.finalord[k];
            atomicAdd(&L.mult[id], 1u);
            atomicMin(&L.firstp[id], k);
        }
        __syncthreads();
        for (int lv = kLevels - 1; lv >= 0; --lv) {
            const uint32_t np = L.np[lv];
            for (uint32_t j = tid; j < np; j += kTThreads) {
                const uint32_t id = pkg_id((uint32_t)lv, j), m = L.mult[id];
                if (!m) continue;
                const uint32_t f = L.firstp[id], pr = L.pair[lv][j];
                const uint32_t c0 = pr >> 16, c1 = pr & 0xFFFFu;
                atomicAdd(&L.mult[c0], m);
                atomicMin(&L.firstp[c0], f);
                atomicAdd(&L.mult[c1], m);
                atomicMin(&L.firstp[c1], f);
            }
            __syncthreads();
        }
    }

    TSTAMP(6);
    // ---- 4. code_lengths' insertion order (first final package, then symbol) and its
    // iteration order; lengths, preventOnlyOnesCode, canonical codes ----
    for (uint32_t i = tid; i < n; i += kTThreads) {  // insertion rank of leaf i
        const uint32_t f = L.firstp[i], s = L.leafsym[i];
        uint32_t r = 0;
        for (uint32_t x = 0; x < n; ++x) {
            const uint32_t fx = L.firstp[x];
            r += (fx < f || (fx == f && L.leafsym[x] < s)) ? 1u : 0u;
        }
        L.arr[r] = i;  // (L.arr: the leaf inserted r-th; map_order reuses arr, so move it)
    }
    __syncthreads();
    for (uint32_t r = tid; r < n; r += kTThreads) {
        L.order[r] = L.arr[r];                 // leaf of insertion r
        L.sl[r] = L.leafsym[L.arr[r]];         // its key
    }
    __syncthreads();
    map_order(L, L.sl, n, L.order2, tid);      // order2[m] = insertion rank of the m-th iterated
    for (uint32_t m = tid; m < n; m += kTThreads) L.items[m] = L.order[L.order2[m]];  // leaf iterated m-th
    __syncthreads();
    // the longest length's last symbol (in iteration order) moves one level deeper
    if (tid == 0) {
        uint32_t lmax = 0, mlast = 0;
        for (uint32_t m = 0; m < n; ++m) {
            const uint32_t l = L.mult[L.items[m]];
            if (l >= lmax) { lmax = l; mlast = m; }
        }
        for (int l = 0; l < 18; ++l) L.bits[l] = 0;
        for (uint32_t m = 0; m < n; ++m) {
            const uint32_t leaf = L.items[m];
            const uint32_t l = L.mult[leaf] + (m == mlast ? 1u : 0u);
            L.len[m] = l;
            L.bits[l] += 1;
        }
    }
    __syncthreads();
    // canonical codes (generateCodes, Huffman.cpp:50-66): lengths ascending, each length
    // in iteration order; the DHT lists the symbols in the same order
    for (uint32_t m = tid; m < n; m += kTThreads) {
        const uint32_t l = L.len[m];
        uint32_t code = 0, before = 0;  // first code of length l; symbols of shorter lengths
        for (uint32_t k = 1; k < l; ++k) {
            code = (code + L.bits[k]) << 1;
            before += L.bits[k];
        }
        uint32_t pos = 0;  // earlier symbols of the same length
        for (uint32_t x = 0; x < m; ++x) pos += L.len[x] == l ? 1u : 0u;
        const uint32_t s = L.leafsym[L.items[m]];
        tab[s] = (l << 16) | ((code + pos) & 0xFFFFu);
        dht[17 + before + pos] = (uint8_t)s;
    }
    if (tid == 0) {
        dht[0] = (uint8_t)(((t & 1) << 4) | (t >> 1));
        for (int l = 1; l <= 16; ++l) dht[l] = (uint8_t)L.bits[l];
        *nsym = n;
    }
    TSTAMP(7);
#undef TSTAMP
}

}  // namespace

size_t huff_tables_lds_bytes() { return sizeof(TabLds); }

hipError_t launch_huff_tables(const TabArgs& a, uint32_t sets, hipStream_t s) {
    static bool attr = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void*>(huff_tables_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(TabLds)) == hipSuccess;
    }();
    if (!attr) return hipErrorInvalidValue;
    hipLaunchKernelGGL(huff_tables_kernel, dim3(4, sets), dim3(kTThreads), sizeof(TabLds), s, a);
    return hipGetLastError();
}

}  // namespace jpge
