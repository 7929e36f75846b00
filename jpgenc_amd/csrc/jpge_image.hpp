// C++ facade with the reference's entry points (include/Image.hpp:28-115), built
// purely on the C ABI in include/jpge.h.  A jpgEnc user switches by replacing
//     #include "Image.hpp"            ->  #include "jpge_image.hpp"
//     auto img = loadPPM(path);       ->  auto img = jpge::loadPPM(path);
//     img.writeJPEG(out);             (unchanged)
// Errors surface as std::runtime_error, the reference's convention (Image.cpp:428,450).
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "jpge.h"

namespace jpge {

class Image {
  public:
    enum ColorSpace { RGB, YCbCr };
    enum SubsamplingMode { S444, S422, S411, S420, S420_m, S420_lm };  // Image.hpp:44-52
    enum DCTMode { Simple, Matrix, Arai };

    Image(uint32_t w, uint32_t h, std::vector<uint8_t> rgb, int maxval);

    // Image::writeJPEG(std::string) — Image.hpp:92.  Quality 50 is the reference's
    // only setting; other qualities scale the same tables (IJG rule).
    void writeJPEG(const std::string& file, int quality = 50) const;
    std::vector<uint8_t> encode(int quality = 50) const;

    // applyDCT(Arai) + applyQuantization(qy, qc) (Image.hpp:81-82) fused on the GPU;
    // results are the quantised planes QY/QCb/QCr (block raster, natural order).
    void applyDCTAndQuantization(const uint8_t qy[64], const uint8_t qc[64]);
    const std::vector<int16_t>& QY() const { return qy_; }
    const std::vector<int16_t>& QCb() const { return qcb_; }
    const std::vector<int16_t>& QCr() const { return qcr_; }

    // geometry fields with the reference's names (Image.hpp:101-103)
    uint32_t width, height;            // padded to multiples of 16
    uint32_t real_width, real_height;  // as in the PPM
    uint32_t subsample_width, subsample_height;
    int maxval;
    const std::vector<uint8_t>& rgb() const { return rgb_; }

  private:
    std::vector<uint8_t> rgb_;
    std::vector<int16_t> qy_, qcb_, qcr_;
};

// loadPPM (Image.hpp:28): P3 / P6, throws std::runtime_error on failure.
Image loadPPM(const std::string& path);

// The process-wide context the facade encodes with (device from JPGE_DEVICE, default 0).
jpge_ctx* default_context();

}  // namespace jpge
