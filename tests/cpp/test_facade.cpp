// The drop-in facade (jpgenc_amd/csrc/jpge_image.hpp) under the reference's own unit
// tests, restated as known-answer checks with the reference's values and compiled
// against the facade exactly as reference code would be (global names, no edits to
// the calls):
//   cpu   CodingTest.cpp:5-162 (RLE_AC, encode_category, getCategoryAndCode),
//         BitstreamGenericTest.cpp:11-221 (bit order, fill, compare, extract, LSB
//         mode), DctTest.cpp:86-158 (zigzag, quantize), ImageTest.cpp:7-45 (loadPPM
//         with padding), Huffman text round trips (Huffman.cpp:3-146)
//   gpu   ImageTest.cpp:47-73 (convertToColorSpace), :75-199 (applySubsampling, all
//         modes), :347-353 (applyDCT Matrix), the stage chain of writeJPEG, writeJPEG
//         on the fused and the plane paths (files for the pytest driver to compare
//         with the oracle), and two threads encoding different images at once.
// Usage: test_facade cpu <ppm dir> | test_facade gpu <ppm dir> <out dir>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "jpge_image.hpp"

static int g_fail = 0, g_checks = 0;
#define CHECK(cond)                                                                    \
    do {                                                                               \
        ++g_checks;                                                                    \
        if (!(cond)) {                                                                 \
            ++g_fail;                                                                  \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);        \
        }                                                                              \
    } while (0)
#define CHECK_EQUAL(a, b) CHECK((a) == (b))
// unittest.hpp:12-13: the reference's tolerance for its floating-point checks
#define CHECK_CLOSE(a, b) CHECK(std::fabs((double)(a) - (double)(b)) < 1e-5)

static std::string g_res;
static std::string res(const char* name) { return g_res + "/" + name; }

// ---------------------------------------------------------------- cpu

// CodingTest.cpp:5-68
static void rle_ac_vector() {
    std::vector<int> data(64, 0), zero_end(64, 0);
    data[0] = zero_end[0] = -111;
    data[1] = zero_end[1] = 57;
    data[20] = zero_end[20] = 3;
    data[25] = zero_end[25] = -2;
    data[63] = -2;
    const std::vector<RLE_PAIR> want{RLE_PAIR(0, -111), RLE_PAIR(0, 57), RLE_PAIR(15, 0), RLE_PAIR(2, 3),
                                     RLE_PAIR(4, -2),   RLE_PAIR(15, 0), RLE_PAIR(15, 0), RLE_PAIR(5, -2)};
    const std::vector<RLE_PAIR> want_zero_end{RLE_PAIR(0, -111), RLE_PAIR(0, 57), RLE_PAIR(15, 0),
                                              RLE_PAIR(2, 3),    RLE_PAIR(4, -2), RLE_PAIR(0, 0)};
    auto rle = RLE_AC(data);
    CHECK(want == rle);
    CHECK(want_zero_end == RLE_AC(zero_end));

    auto coded = encode_category(rle);
    std::vector<Category_Code> want_coding;
    want_coding.emplace_back(7, Bitstream(16, 7));
    want_coding.emplace_back(6, Bitstream(57, 6));
    want_coding.emplace_back(240, Bitstream());
    want_coding.emplace_back(34, Bitstream(3, 2));
    want_coding.emplace_back(66, Bitstream(1, 2));
    want_coding.emplace_back(240, Bitstream());
    want_coding.emplace_back(240, Bitstream());
    want_coding.emplace_back(82, Bitstream(1, 2));
    CHECK(want_coding == coded);
}

// CodingTest.cpp:70-131
static void rle_ac_matrix() {
    std::vector<int> data(64, 0), zero_end(64, 0);
    data[0] = zero_end[0] = -111;
    data[1] = zero_end[1] = 57;
    data[20] = zero_end[20] = 3;
    data[25] = zero_end[25] = -2;
    data[63] = -2;
    auto m = from_vector(data);
    auto mz = from_vector(zero_end);
    const std::vector<RLE_PAIR> want{RLE_PAIR(0, -111), RLE_PAIR(0, 57), RLE_PAIR(9, -2), RLE_PAIR(13, 3),
                                     RLE_PAIR(15, 0),   RLE_PAIR(15, 0), RLE_PAIR(5, -2)};
    const std::vector<RLE_PAIR> want_zero_end{RLE_PAIR(0, -111), RLE_PAIR(0, 57), RLE_PAIR(9, -2), RLE_PAIR(13, 3),
                                              RLE_PAIR(0, 0)};
    CHECK(want == RLE_AC(m));
    CHECK(want_zero_end == RLE_AC(mz));
}

// CodingTest.cpp:133-162
static void category_and_code() {
    short cat = 0;
    CHECK(std::make_pair(cat, Bitstream()) == getCategoryAndCode(0));
    const struct {
        short cat;
        int value;
        uint32_t bits;
    } kat[] = {{1, -1, 0},       {1, 1, 1},        {2, -3, 0},        {2, -2, 1},      {2, 2, 2},
               {2, 3, 3},        {3, -7, 0},       {3, -6, 1},        {3, -4, 3},      {3, 4, 4},
               {3, 6, 6},        {3, 7, 7},        {10, -1023, 0},    {10, -1022, 1},  {10, -512, 511},
               {10, 512, 512},   {10, 1022, 1022}, {10, 1023, 1023}};
    for (const auto& k : kat) CHECK(std::make_pair(k.cat, Bitstream(k.bits, k.cat)) == getCategoryAndCode(k.value));
    // the two-output form (Coding.hpp:197-230) agrees
    short c2 = -1;
    Bitstream b2;
    getCategoryAndCode(-512, c2, b2);
    CHECK(c2 == 10 && b2 == Bitstream(511, 10));
}

// BitstreamGenericTest.cpp:11-221
static void bitstreams() {
    Bitstream def;
    CHECK_EQUAL(def.size(), 0u);
    Bitstream b0{1, 0, 0, 1, 1, 1, 1, 0, 0, 1};
    CHECK(b0[0] == true);
    CHECK(b0[2] == false);
    CHECK(b0[4] == true);
    CHECK(b0[8] == false);
    CHECK(b0[9] == true);
    CHECK_EQUAL(b0.size(), 10u);
    b0[0] = false;
    b0[8] = 1;
    CHECK(b0[0] == false);
    CHECK(b0[8] == true);
    b0 << Bits{1, 0, 0, 1};
    CHECK(b0[10] == true && b0[11] == false && b0[12] == false && b0[13] == true);
    CHECK_EQUAL(b0.size(), 14u);
    b0 << false << true << true << true;
    CHECK(b0[14] == false && b0[15] == true && b0[16] == true && b0[17] == true);
    CHECK_EQUAL(b0.size(), 18u);

    auto b8 = Bitstream8();
    b8.push_back(0x34000000, 6);  // 001101
    CHECK(b8[0] == 0 && b8[1] == 0 && b8[2] == 1 && b8[3] == 1 && b8[4] == 0 && b8[5] == 1);

    auto b1 = Bitstream8{1, 0, 1, 1, 0, 0};
    auto b2 = Bitstream8{0, 0, 1, 1, 0, 0};
    b1 << b2;
    CHECK_EQUAL(b1.size(), 12u);
    CHECK_EQUAL(b1.extractT<uint16_t>((uint8_t)b1.size(), 0), 0xB0C0);

    {  // written and read back through a stream of blocks
        Bitstream bits;
        bool val = false;
        for (int x = 0; x < 1000; ++x) {
            if (!(x % 4)) val = !val;
            bits << val;
        }
        CHECK_EQUAL(bits.size(), 1000u);
        std::stringstream ss;
        ss << bits;
        Bitstream in;
        ss >> in;
        CHECK(in[0] == true && in[3] == true && in[4] == false && in[7] == false);
        CHECK(in[8] == true && in[11] == true && in[12] == false);
        CHECK_EQUAL(in.size(), 1000u);  // (1000 bits are whole bytes)
    }

    Bitstream8 bs{1, 0, 0, 1};
    bs.fill();
    CHECK(bs[0] == true && bs[1] == false && bs[2] == false && bs[3] == true);
    CHECK(bs[4] == true && bs[5] == true && bs[6] == true && bs[7] == true);
    bs << Bits{0, 1};
    CHECK(bs[8] == false && bs[9] == true);
    Bitstream8 bs2{0, 0, 0, 0, 0, 0, 0, 0};
    bs2.fill();
    CHECK_EQUAL(bs2.size(), 8u);

    Bitstream8 bs3{1, 1, 0, 0, 1, 1, 0, 0, 1, 1, 0, 0, 1, 1};
    Bitstream8 bs4{1, 1, 0, 0, 1, 1, 0, 0, 1, 1, 0, 0, 1, 1};
    Bitstream8 bs5{1, 1, 0, 0, 1, 1, 0, 0, 1, 1, 0, 0, 1, 0};
    Bitstream8 bs6{1, 1, 0, 0, 1, 1, 0, 0, 1, 1, 0, 0, 1, 1, 0};
    CHECK(bs3 == bs4);
    CHECK(bs3 != bs5);
    CHECK(bs3 != bs6);

    auto b = Bitstream8{1, 0, 0, 1, 1, 1};
    CHECK_EQUAL(b.extractT<uint16_t>(3, 0), 0x8000);
    CHECK_EQUAL(b.extractT<uint16_t>(4, 2), 0x7000);
    b = Bitstream8{1, 0, 0, 1, 1, 1, 0, 0, 1, 0, 1};
    CHECK_EQUAL(b.extractT<uint16_t>(11, 0), 0x9CA0);
    CHECK_EQUAL(b.extractT<uint16_t>(5, 6), 0x2800);
    CHECK_EQUAL(b.extractT<uint8_t>(4, 1), 0x30);
    CHECK_EQUAL(b.extractT<uint16_t>((uint8_t)b.size(), 0), 0x9CA0);
    CHECK_EQUAL(b.extractT<uint32_t>(5, 6), 0x28000000u);
    CHECK_EQUAL(b.extractT<uint64_t>(6, 3), 0xE400000000000000ull);

    auto lsb = Bitstream8();
    lsb.push_back_LSB_mode(4, 4);  // 0100
    CHECK_EQUAL(lsb.extractT<uint8_t>(4, 0), 0x40);

    // stuffing on output (BitstreamGeneric.hpp:213-224)
    Bitstream ff;
    ff.push_back(0xFF000000u, 8);
    ff.push_back(0x12000000u, 8);
    std::ostringstream os;
    os << ff;
    CHECK(os.str() == std::string("\xFF\x00\x12", 3));
}

// DctTest.cpp:86-158
static void zigzag_and_quantize() {
    std::vector<int> nat(64);
    for (int i = 0; i < 64; ++i) nat[i] = i + 1;
    auto v = zigzag(from_vector(nat));
    const std::vector<int> want_zz{1,  2,  9,  17, 10, 3,  4,  11, 18, 25, 33, 26, 19, 12, 5,  6,
                                   13, 20, 27, 34, 41, 49, 42, 35, 28, 21, 14, 7,  8,  15, 22, 29,
                                   36, 43, 50, 57, 58, 51, 44, 37, 30, 23, 16, 24, 31, 38, 45, 52,
                                   59, 60, 53, 46, 39, 32, 40, 47, 54, 61, 62, 55, 48, 56, 63, 64};
    CHECK(v == want_zz);
    for (int i = 0; i < 64; ++i) CHECK_EQUAL(zigzag(i) + 1, v[i]);
    const auto y_table = from_vector<int>({16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                                           14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                                           18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                                           49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99});
    auto input = from_vector<PixelDataType>({581, -144, 56,  17,  15, -7,  25, -9, -242, 133, -48, 42, -2, -7, 13, -4,
                                             108, -18,  -40, 71,  -33, 12, 6,  -10, -56, -93, 48, 19, -8, 7,  6,  -2,
                                             -17, 9,    7,   -23, -3, -10, 5,  3,  4,    9,   -4,  -5, 2,  2,  -7, 3,
                                             -9,  7,    8,   -6,  5,  12,  2,  -5, -9,   -4,  -2,  -3, 6,  1,  -1, -1});
    auto true_result = from_vector<int>({36, -13, 6,  1, 1,  0, 0, 0, -20, 11, -3, 2, 0, 0, 0, 0, 8, -1, -3, 3, -1, 0,
                                         0,  0,   -4, -5, 2, 1, 0, 0, 0,   0,  -1, 0, 0, 0, 0, 0, 0, 0,  0,  0, 0,  0,
                                         0,  0,   0,  0, 0,  0, 0, 0, 0,   0,  0,  0, 0, 0, 0, 0, 0, 0,  0,  0});
    CHECK(quantize(input, y_table) == true_result);
}

// ImageTest.cpp:7-45 (maxval 15, 4x4 padded to 16x16 by edge replication)
static void image_loading() {
    auto image = loadPPM(res("tester_p3.ppm"));
    CHECK(image.R(0, 0) == 0 && image.G(0, 0) == 0 && image.B(0, 0) == 0);
    CHECK(image.R(0, 3) == 255 && image.G(0, 3) == 0 && image.B(0, 3) == 255);
    CHECK(image.R(2, 2) == 0 && image.G(2, 2) == 255 && image.B(2, 2) == 119);
    CHECK(image.R(15, 0) == 255 && image.G(15, 0) == 0 && image.B(15, 0) == 255);
    CHECK(image.R(0, 15) == 255 && image.G(0, 15) == 0 && image.B(0, 15) == 255);
    CHECK(image.R(1, 15) == 0 && image.G(1, 15) == 0 && image.B(1, 15) == 0);
    CHECK(image.R(15, 1) == 0 && image.G(15, 1) == 0 && image.B(15, 1) == 0);
    CHECK(image.R(15, 15) == 0 && image.G(15, 15) == 0 && image.B(15, 15) == 0);
    CHECK_EQUAL(image.width, 16u);
    CHECK_EQUAL(image.real_width, 4u);
    CHECK(!image.isFrame());  // non-const plane access ends the frame
    auto fresh = loadPPM(res("tester_p3.ppm"));
    CHECK(fresh.isFrame());
    bool threw = false;
    try {
        loadPPM(res("no_such_file.ppm"));
    } catch (const std::runtime_error&) {
        threw = true;
    }
    CHECK(threw);
}

// Huffman.hpp / Huffman.cpp: the code of a text, encode and decode round trip
static void huffman() {
    const std::vector<int> text{1, 2, 2, 5, 5, 5, 5, 7, 7, 3, 1, 5, 22, 33, 5, 2};
    auto hc = generateHuffmanCode(text);
    CHECK_EQUAL(hc.second.size(), 17u);
    size_t nsym = 0;
    for (const auto& l : hc.second) nsym += l.size();
    CHECK_EQUAL(nsym, hc.first.size());
    auto bits = huffmanEncode(text, hc.first);
    CHECK(huffmanDecode(bits, hc.first) == text);
    auto one = generateHuffmanCode({9, 9, 9});  // one symbol: code "0" (Huffman.cpp:17-25)
    CHECK(one.first[9].length == 1 && one.first[9].code == 0u);
    CHECK(one.second[1] == std::vector<int>{9});
}

// ---------------------------------------------------------------- gpu

// ImageTest.cpp:47-73
static void color_conversion() {
    auto image = loadPPM(res("tester_p3.ppm"));
    auto ycc = image.convertToColorSpace(Image::YCbCr);
    CHECK_CLOSE(ycc.Y(0, 3), -22.685);
    CHECK_CLOSE(ycc.Cb(0, 3), 84.4815);
    CHECK_CLOSE(ycc.Cr(0, 3), 106.7685);
    CHECK_CLOSE(ycc.Y(1, 1), 35.251);
    CHECK_CLOSE(ycc.Cb(1, 1), -24.956);
    CHECK_CLOSE(ycc.Cr(1, 1), -116.417698);
    ycc = image.convertToColorSpace(Image::YCbCr);
    CHECK_CLOSE(ycc.Y(0, 3), -22.685);
    CHECK_CLOSE(ycc.Cb(0, 3), 84.4815);
    CHECK_CLOSE(ycc.Cr(0, 3), 106.7685);
    auto rgb = image.convertToColorSpace(Image::RGB);
    CHECK_CLOSE(rgb.R(0, 3), 255);
    CHECK_CLOSE(rgb.G(0, 3), 0);
    CHECK_CLOSE(rgb.B(0, 3), 255);
    CHECK_CLOSE(rgb.R(1, 1), 0);
    CHECK_CLOSE(rgb.G(1, 1), 255);
    CHECK_CLOSE(rgb.B(1, 1), 119);
    // and back: YCbCr -> RGB, the reference's formula as written (Image.cpp:164-171: the
    // chroma planes are offset by +128, not recentred; tests/test_gpu_planes.py pins
    // the plane kernel to it bit for bit)
    auto back = ycc.convertToColorSpace(Image::RGB);
    const double y = ycc.Y(1, 1) + 128, cb = ycc.Cb(1, 1) + 128, cr = ycc.Cr(1, 1) + 128;
    CHECK_EQUAL(back.G(1, 1), (1.f * y + -.344f * cb + -.714f * cr));
    CHECK(back.colorSpace() == Image::RGB);
}

// ImageTest.cpp:75-199
static void subsampling() {
    auto orig = loadPPM(res("tester_p3.ppm"));
    {
        auto image = orig;
        image.applySubsampling(Image::S444);
        CHECK_EQUAL(image.B.size2(), 16u);
        CHECK_EQUAL(image.B.size1(), 16u);
    }
    {
        auto image = orig;
        image.applySubsampling(Image::S422);
        CHECK_EQUAL(image.B.size2(), 8u);
        CHECK_EQUAL(image.B.size1(), 16u);
        CHECK_EQUAL(image.B(2, 0), 0);
        CHECK_EQUAL(image.B(2, 1), 119);
        CHECK_EQUAL(image.B(3, 0), 255);
        CHECK_EQUAL(image.B(3, 1), 0);
        CHECK_EQUAL(image.G(2, 0), 0);
        CHECK_EQUAL(image.G(2, 1), 255);
        CHECK_EQUAL(image.G(3, 0), 0);
    }
    {
        auto image = orig;
        image.applySubsampling(Image::S411);
        CHECK_EQUAL(image.B.size2(), 4u);
        CHECK_EQUAL(image.B.size1(), 16u);
        CHECK_EQUAL(image.B(2, 0), 0);
        CHECK_EQUAL(image.B(3, 0), 255);
        CHECK_EQUAL(image.G(2, 0), 0);
        CHECK_EQUAL(image.G(3, 0), 0);
    }
    {
        auto image = orig;
        image.applySubsampling(Image::S420);
        CHECK_EQUAL(image.B.size2(), 8u);
        CHECK_EQUAL(image.B.size1(), 8u);
        CHECK_EQUAL(image.B(1, 0), 0);
        CHECK_EQUAL(image.B(1, 1), 119);
        CHECK_EQUAL(image.G(1, 0), 0);
        CHECK_EQUAL(image.G(1, 1), 255);
    }
    {
        auto image = orig;
        image.applySubsampling(Image::S420_m);
        CHECK_EQUAL(image.B.size2(), 8u);
        CHECK_EQUAL(image.B.size1(), 8u);
        CHECK_EQUAL(image.B(0, 0), 29.75);
        CHECK_EQUAL(image.B(1, 0), 63.75);
        CHECK_EQUAL(image.B(0, 1), 63.75);
        CHECK_EQUAL(image.B(1, 1), 29.75);
        CHECK_EQUAL(image.G(0, 0), 63.75);
        CHECK_EQUAL(image.G(1, 0), 0);
        CHECK_EQUAL(image.G(0, 1), 0);
        CHECK_EQUAL(image.G(1, 1), 63.75);
        CHECK_EQUAL(image.subsample_width, 8u);
    }
    {
        auto image = orig;
        image.applySubsampling(Image::S420_lm);
        CHECK_EQUAL(image.B.size2(), 8u);
        CHECK_EQUAL(image.B.size1(), 8u);
        CHECK_EQUAL(image.B(0, 0), 0);
        CHECK_EQUAL(image.B(0, 1), 0);
        CHECK_EQUAL(image.B(1, 0), 127.5);
        CHECK_EQUAL(image.B(1, 1), 59.5);
        CHECK_EQUAL(image.G(0, 0), 0);
        CHECK_EQUAL(image.G(1, 0), 0);
        CHECK_EQUAL(image.G(0, 1), 0);
        CHECK_EQUAL(image.G(1, 1), 127.5);
    }
}

// ImageTest.cpp:347-353 and the stage chain of writeJPEG (Image.cpp:839-927)
static void stages(const std::string& out) {
    {
        auto image = loadPPM(res("tester_p3.ppm"));
        image.applyDCT(Image::Matrix);
        CHECK_EQUAL(image.dctY().size1(), 16u);
    }
    auto image = loadPPM(res("tester_RGB_26x19.ppm"));
    image = image.convertToColorSpace(Image::YCbCr);
    image.applySubsampling(Image::S420_m);
    image.applyDCT(Image::Arai);
    const auto qy = from_vector<int>({16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                                      14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                                      18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                                      49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99});
    const auto qc = from_vector<int>({17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                                      24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                                      99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                                      99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99});
    image.applyQuantization(qy, qc);
    // the quantised planes before DC differencing, for the driver (oracle stage coefficients)
    {
        std::ofstream f(out + "/stage_q.txt");
        for (const auto* m : {&image.qY(), &image.qCb(), &image.qCr()}) {
            f << m->size1() << " " << m->size2();
            for (int v : m->data()) f << " " << v;
            f << "\n";
        }
    }
    image.applyDCdifferenceCoding();
    image.doRLEandCategoryCoding();
    // symbol texts (Image.cpp:888-906) -> tables -> emission, as writeJPEG does
    std::vector<int> ydc, yac, cdc, cac;
    for (const auto& d : image.categoryCodeY().data()) {
        ydc.push_back(d[0].symbol);
        for (size_t k = 1; k < d.size(); ++k) yac.push_back(d[k].symbol);
    }
    for (const auto* cc : {&image.categoryCodeCb(), &image.categoryCodeCr()})
        for (const auto& d : cc->data()) {
            cdc.push_back(d[0].symbol);
            for (size_t k = 1; k < d.size(); ++k) cac.push_back(d[k].symbol);
        }
    auto hydc = generateHuffmanCode(ydc), hyac = generateHuffmanCode(yac);
    auto hcdc = generateHuffmanCode(cdc), hcac = generateHuffmanCode(cac);
    image.doHuffmanEncoding(hydc.first, hyac.first, hcdc.first, hcac.first);
    // MCU interleave + fill (Image.cpp:957-970): the entropy-coded segment
    Bitstream stream;
    const auto& by = image.bitstreamY();
    const auto &bcb = image.bitstreamCb(), &bcr = image.bitstreamCr();
    for (size_t i = 0; i < bcb.size1(); ++i)
        for (size_t j = 0; j < bcb.size2(); ++j) {
            stream << by(2 * i, 2 * j) << by(2 * i, 2 * j + 1) << by(2 * i + 1, 2 * j) << by(2 * i + 1, 2 * j + 1);
            stream << bcb(i, j) << bcr(i, j);
        }
    stream.fill();
    std::ofstream f(out + "/stage_entropy.bin", std::ios::binary);
    f << stream;
}

static void write_files(const std::string& out) {
    // the fused path (the loaded frame) and the plane path (a plane written)
    for (const char* name : {"tester_p3.ppm", "tester_RGB_26x19.ppm", "tester_text_32x32.ppm", "tester_p6.ppm"}) {
        auto a = loadPPM(res(name));
        CHECK(a.isFrame());
        a.writeJPEG(out + "/" + name + ".frame.jpg");
        auto b = loadPPM(res(name));
        b.R(0, 0) = b.R(0, 0);  // a write access: the planes are now the image
        CHECK(!b.isFrame());
        b.writeJPEG(out + "/" + name + ".planes.jpg");
        CHECK(b.Y.size1() == 0);  // consumed, as the reference's
    }
    // an Image built from scratch (Image.hpp:64), in both colour spaces
    Image img(48, 32, Image::RGB);
    for (uint y = 0; y < 32; ++y)
        for (uint x = 0; x < 48; ++x) {
            img.R(y, x) = (x * 5) % 256;
            img.G(y, x) = (y * 7) % 256;
            img.B(y, x) = ((x + y) * 3) % 256;
        }
    auto ycc = img.convertToColorSpace(Image::YCbCr);
    img.writeJPEG(out + "/built_rgb.jpg");
    ycc.writeJPEG(out + "/built_ycc.jpg");
    auto q90 = loadPPM(res("tester_RGB_26x19.ppm"));
    q90.writeJPEG(out + "/tester_RGB_26x19.q90.jpg", 90);
}

// Images on two threads at once share the default context
static void two_threads(const std::string& out) {
    std::vector<uint8_t> r1, r2;
    auto work = [](const char* name, int reps, std::vector<uint8_t>* o) {
        for (int i = 0; i < reps; ++i) {
            auto img = loadPPM(g_res + "/" + name);
            auto bytes = img.encode(75);
            if (i == 0) *o = bytes;
            else if (bytes != *o) o->clear();  // (any difference between repetitions)
        }
    };
    std::thread t1(work, "tester_text_32x32.ppm", 40, &r1);
    std::thread t2(work, "tester_RGB_26x19.ppm", 40, &r2);
    t1.join();
    t2.join();
    CHECK(!r1.empty() && !r2.empty());
    std::ofstream(out + "/thread_a.jpg", std::ios::binary).write((const char*)r1.data(), (std::streamsize)r1.size());
    std::ofstream(out + "/thread_b.jpg", std::ios::binary).write((const char*)r2.data(), (std::streamsize)r2.size());
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: test_facade cpu <ppm dir> | gpu <ppm dir> <out dir>\n");
        return 2;
    }
    const std::string mode = argv[1];
    g_res = argv[2];
    try {
        if (mode == "cpu") {
            rle_ac_vector();
            rle_ac_matrix();
            category_and_code();
            bitstreams();
            zigzag_and_quantize();
            image_loading();
            huffman();
        } else if (mode == "gpu" && argc >= 4) {
            color_conversion();
            subsampling();
            stages(argv[3]);
            write_files(argv[3]);
            two_threads(argv[3]);
        } else {
            return 2;
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "exception: %s\n", e.what());
        return 3;
    }
    std::printf("%d checks, %d failed\n", g_checks, g_fail);
    return g_fail ? 1 : 0;
}
