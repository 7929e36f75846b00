// jpgenc — CLI with the reference's contract (src/main.cpp:8-32):
//   jpgenc <in.ppm> [out.jpg]      default output "noname.jpg"; no arguments
//                                  prints "No filename was written" and exits 0.
// Extensions: -q <1..100> (IJG-scaled tables, 50 = reference), JPGE_DEVICE=<n>;
//   --gpus N / --devices a,b,...   one image row-striped over a device group
//                                  (jpge_group_encode_striped: RCCL between distinct
//                                  devices), e.g. a 16384^2 frame over 8 GPUs;
//   --restart M                    restart interval in MCUs (DRI/RSTn).
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <iterator>
#include <sstream>
#include <string>
#include <vector>

#include "jpge_image.hpp"

namespace {
int striped(const std::vector<int>& devs, const std::string& in, const std::string& out, int quality,
            uint32_t restart) {
    std::ifstream f(in, std::ios::binary);
    if (!f.is_open()) throw std::runtime_error("Failed to open \"" + in + "\"");
    std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    uint32_t w = 0, h = 0;
    int mv = 0;
    jpge::detail::check(jpge_ppm_info(buf.data(), buf.size(), &w, &h, &mv), "loadPPM");
    std::vector<uint8_t> rgb((size_t)w * h * 3);
    jpge::detail::check(jpge_parse_ppm(buf.data(), buf.size(), rgb.data(), rgb.size(), &w, &h, &mv), "loadPPM");
    uint8_t qy[64], qc[64];
    jpge::detail::check(jpge_quality_tables(quality, qy, qc), "quality");
    jpge_group* g = nullptr;
    jpge::detail::check(jpge_group_open((int)devs.size(), devs.data(), 1, &g), "jpge_group_open");
    std::vector<uint8_t> jpg(jpge_max_jpeg_bytes(w, h));
    size_t len = 0;
    int st = jpge_group_set_restart_interval(g, restart);
    if (!st) st = jpge_group_encode_striped(g, rgb.data(), w, h, 0, mv, qy, qc, jpg.data(), jpg.size(), &len);
    jpge_group_close(g);
    jpge::detail::check(st, "jpge_group_encode_striped");
    std::ofstream o(out, std::ios::binary);
    if (!o.is_open()) throw std::runtime_error("Failed to open \"" + out + "\"");
    o.write(reinterpret_cast<const char*>(jpg.data()), (std::streamsize)len);
    return 0;
}
}  // namespace

int main(int argc, char* argv[]) {
    std::vector<std::string> pos;
    std::vector<int> devs;
    int quality = 50;
    uint32_t restart = 0;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "-q") && i + 1 < argc) {
            quality = std::atoi(argv[++i]);
        } else if (!std::strcmp(argv[i], "--gpus") && i + 1 < argc) {
            const int n = std::atoi(argv[++i]);
            devs.clear();
            for (int d = 0; d < n; ++d) devs.push_back(d);
        } else if (!std::strcmp(argv[i], "--devices") && i + 1 < argc) {
            devs.clear();
            std::stringstream ss(argv[++i]);
            std::string t;
            while (std::getline(ss, t, ',')) devs.push_back(std::atoi(t.c_str()));
        } else if (!std::strcmp(argv[i], "--restart") && i + 1 < argc) {
            restart = (uint32_t)std::strtoul(argv[++i], nullptr, 10);
        } else {
            pos.emplace_back(argv[i]);
        }
    }
    if (pos.empty()) {
        std::cout << "No filename was written" << std::endl;
        return 0;
    }
    const std::string jpg = pos.size() < 2 ? "noname.jpg" : pos[1];
    try {
        if (!devs.empty()) return striped(devs, pos[0], jpg, quality, restart);
        auto img = jpge::loadPPM(pos[0]);
        if (restart) jpge::detail::check(jpge_set_restart_interval(jpge::default_context(), restart), "restart");
        img.writeJPEG(jpg, quality);
    } catch (const std::exception& e) {
        std::cerr << "jpgenc: " << e.what() << std::endl;
        return 1;
    }
    return 0;
}
