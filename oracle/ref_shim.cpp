// TEST INFRASTRUCTURE ONLY — a ctypes harness around the reference's OWN
// Huffman table builder and Bitstream class, compiled unmodified from
// /root/reference (src/Huffman.cpp, include/Huffman.hpp,
// include/BitstreamGeneric.hpp) by oracle/Makefile into oracle/_ref/.
// Nothing here is product code and nothing is copied from the reference: this
// file only calls the reference functions and flattens their results.
#include <cstdint>
#include <sstream>
#include <string>
#include <vector>

#include "Huffman.hpp"

extern "C" {

// generateHuffmanCode (Huffman.cpp:3-35) on an int text.  Emits the DHT-order
// (SymbolsPerLength) flattening and the code value of each symbol.
int ref_huffman(const int* text, int n, int* dht_syms, int* dht_lens, uint32_t* codes) {
    std::vector<int> t(text, text + n);
    auto res = generateHuffmanCode(t);
    int k = 0;
    for (size_t len = 1; len < res.second.size(); ++len)
        for (int s : res.second[len]) {
            const Code& c = res.first[s];
            dht_syms[k] = s;
            dht_lens[k] = (int)len;
            codes[k] = c.length ? (c.code >> (32 - c.length)) : 0u;
            ++k;
        }
    return k;
}

// package_merge (Huffman.hpp:114-174) directly, for the PackageMergeTest shape.
int ref_package_merge(const int* syms, const int* freqs, int n, int limit, int* out_syms, int* out_lens) {
    std::vector<Symbol> v;
    for (int i = 0; i < n; ++i) v.emplace_back(syms[i], freqs[i]);
    auto r = package_merge(v, limit);
    int k = 0;
    for (size_t len = 0; len < r.size(); ++len)
        for (int s : r[len]) { out_syms[k] = s; out_lens[k] = (int)len; ++k; }
    return k;
}

// Bitstream (BitstreamGeneric.hpp): mode 0 appends `nbits` of vals[i] via
// push_back(MSB-aligned code, len) as doHuffmanEncoding does with Huffman codes
// (Image.cpp:758); mode 1 appends a Bitstream(vals[i], nbits) built in LSB mode
// via operator<<(Bitstream&), as it does with category codes (Image.cpp:759).
// Then fill() and the stuffing ostream<<.  Returns the stuffed byte count.
int64_t ref_pack_bits(const uint32_t* vals, const int* nbits, const int* modes, int n, int do_fill,
                      uint8_t* out, int64_t cap, int64_t* raw_bits) {
    Bitstream s;
    for (int i = 0; i < n; ++i) {
        if (nbits[i] == 0) continue;
        if (modes[i] == 0) {
            s.push_back(vals[i] << (32 - nbits[i]), nbits[i]);
        } else {
            Bitstream c(vals[i], nbits[i]);
            s << c;
        }
    }
    if (do_fill) s.fill();
    *raw_bits = s.size();
    std::ostringstream os;
    os << s;
    std::string b = os.str();
    if ((int64_t)b.size() > cap) return -(int64_t)b.size();
    std::copy(b.begin(), b.end(), out);
    return (int64_t)b.size();
}

// The reference's own round trip (HuffmanTest.cpp:65-85): generateHuffmanCode,
// huffmanEncode (Huffman.cpp:69-76) and huffmanDecode (Huffman.cpp:91-146).  bits
// receives the encoded stream MSB-first (cap bytes, zeroed by the caller); decoded
// the decoded text (n entries).  Returns the bit count.
int64_t ref_huffman_roundtrip(const int* text, int n, uint8_t* bits, int64_t cap, int* decoded) {
    std::vector<int> t(text, text + n);
    auto res = generateHuffmanCode(t);
    Bitstream enc = huffmanEncode(t, res.first);
    const int64_t nb = (int64_t)enc.size();
    if ((nb + 7) / 8 > cap) return -1;
    for (int64_t i = 0; i < nb; ++i)
        if (enc.extract(1, (unsigned)i) >> 31) bits[i >> 3] |= (uint8_t)(0x80u >> (i & 7));
    std::vector<int> dec = huffmanDecode(enc, res.first);
    for (size_t i = 0; i < dec.size() && i < (size_t)n; ++i) decoded[i] = dec[i];
    return nb;
}

}  // extern "C"
