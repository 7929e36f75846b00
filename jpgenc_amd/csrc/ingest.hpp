// PPM files -> .jpg files through the encoder, pipelined by groups of frames
// (read + parse into pinned memory | H2D + kernels | D2H + write); see ingest.cpp.
#pragma once
#include <cstddef>
#include <memory>

#include "encoder.hpp"

namespace jpge {

// Pinned input and device output buffers of the pipeline, kept across calls (a
// context owns one): pinning and device allocation cost far more than a frame.
struct IngestBuffers;
struct IngestBuffersDeleter {
    void operator()(IngestBuffers* b) const;
};

// Encodes in[i] -> out[i] at `quality` (IJG-scaled Annex-K tables, 50 = the
// reference's).  lens[i] / statuses[i] (both optional) get each file's .jpg length
// and status; returns the first failing status.  group: frames per pipeline stage
// (0 = 8, at most 64).
int encode_files(Encoder& enc, std::unique_ptr<IngestBuffers, IngestBuffersDeleter>& bufs, const char* const* in,
                 const char* const* out, int n, int quality, size_t* lens, int* statuses, int group);

}  // namespace jpge
