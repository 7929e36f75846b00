#include "huffman.hpp"

#include <algorithm>
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

void build_code_lengths(const std::vector<std::pair<int, int>>& first_order_counts,
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
            nx.push(Item{a.weight + b.weight, n + (int)kids.size() - 1});
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

bool build_table(const uint32_t counts[256], const uint64_t first_key[256], HuffTable& out) {
    std::vector<std::pair<uint64_t, int>> order;
    for (int s = 0; s < 256; ++s)
        if (counts[s]) order.emplace_back(first_key[s], s);
    if (order.empty()) return false;
    std::sort(order.begin(), order.end());
    std::vector<std::pair<int, int>> fc;
    fc.reserve(order.size());
    for (const auto& o : order) fc.emplace_back(o.second, (int)counts[o.second]);

    std::vector<std::vector<int>> by_len;
    build_code_lengths(fc, by_len);
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
