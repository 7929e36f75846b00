// jpgenc — CLI with the reference's contract (src/main.cpp:8-32):
//   jpgenc <in.ppm> [out.jpg]      default output "noname.jpg"; no arguments
//                                  prints "No filename was written" and exits 0.
// Extensions: -q <1..100> (IJG-scaled tables, 50 = reference), JPGE_DEVICE=<n>.
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "jpge_image.hpp"

int main(int argc, char* argv[]) {
    std::vector<std::string> pos;
    int quality = 50;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "-q") && i + 1 < argc) quality = std::atoi(argv[++i]);
        else pos.emplace_back(argv[i]);
    }
    if (pos.empty()) {
        std::cout << "No filename was written" << std::endl;
        return 0;
    }
    const std::string jpg = pos.size() < 2 ? "noname.jpg" : pos[1];
    try {
        auto img = jpge::loadPPM(pos[0]);
        img.writeJPEG(jpg, quality);
    } catch (const std::exception& e) {
        std::cerr << "jpgenc: " << e.what() << std::endl;
        return 1;
    }
    return 0;
}
