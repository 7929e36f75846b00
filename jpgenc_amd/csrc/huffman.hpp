// Per-image optimal Huffman tables, bit-identical to the reference's
// generateHuffmanCode (src/Huffman.cpp:3-66, include/Huffman.hpp:114-174) as built
// with libstdc++.
//
// The reference's table (DHT symbol order and, through preventOnlyOnesCode, even
// which symbol is demoted) depends on std::unordered_map iteration order and on
// std::priority_queue tie-breaking.  Both are functions of (a) the order in which
// distinct symbols are first inserted and (b) the sequence of weight comparisons,
// so this builder feeds the SAME standard containers with the same insertion
// order and the same comparator, but represents packages as a DAG of node ids
// (no per-package symbol vectors are copied), which makes it O(levels * n).
//
// The GPU supplies, per table, the symbol counts and each symbol's FIRST
// occurrence key (its position in the reference's symbol "text",
// Image.cpp:888-906); sorting by that key reproduces the insertion order.
#pragma once
#include <cstdint>
#include <utility>
#include <vector>

namespace jpge {

struct HuffTable {
    uint8_t bits[17] = {0};       // bits[l] = number of codes of length l (1..16)
    uint8_t huffval[256] = {0};   // symbols in DHT (SymbolsPerLength) order
    int nsym = 0;
    uint32_t code[256] = {0};     // code value (right-aligned) per symbol
    uint8_t len[256] = {0};       // code length per symbol, 0 = symbol has no code
};

// Symbol/count pairs in first-occurrence order -> SymbolsPerLength (17 lists,
// index = code length) and canonical codes, exactly as the reference.
struct GenericCode { uint32_t code; int length; };
void build_code_lengths(const std::vector<std::pair<int, int>>& first_order_counts,
                        std::vector<std::vector<int>>& by_len);
std::vector<std::pair<int, GenericCode>> assign_codes(const std::vector<std::vector<int>>& by_len);

// Byte-symbol table from a 256-bin histogram and first-occurrence keys
// (keys are any totally ordered u64; absent symbols have counts[s] == 0).
// Returns false if every count is zero.
bool build_table(const uint32_t counts[256], const uint64_t first_key[256], HuffTable& out);
// The same with inverted keys (inv_key[s] = ~first_key[s]: the device export's form).
bool build_table_inverted(const uint32_t counts[256], const uint64_t inv_key[256], HuffTable& out);
// The same table through std::unordered_map / std::priority_queue themselves (the
// containers the reference uses; test cross-check of build_table's array emulation).
bool build_table_std(const uint32_t counts[256], const uint64_t first_key[256], HuffTable& out);
void build_code_lengths_std(const std::vector<std::pair<int, int>>& first_order_counts,
                            std::vector<std::vector<int>>& by_len);

// Facade mirror of the reference entry point (Huffman.hpp:53): a symbol text in,
// (symbol -> code) and SymbolsPerLength out.
std::pair<std::vector<std::pair<int, GenericCode>>, std::vector<std::vector<int>>>
generateHuffmanCode(const std::vector<int>& text);

}  // namespace jpge
