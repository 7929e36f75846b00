// a caller whose own exit-time cleanup was registered BEFORE the first
// jpge_open.  Exit handlers run in reverse order of registration, so libjpge's handler
// (live.hpp) releases the context and the group first; the caller's cleanup then
// closes handles the library has already released: those closes must be no-ops, and
// any other call on them must fail cleanly (JPGE_E_ARG), not touch freed memory.
// Run by tests/test_gpu_teardown.py; prints "cleanup ok" from the caller's handler.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "jpge.h"

static jpge_ctx* g_ctx = nullptr;
static jpge_group* g_grp = nullptr;

static void caller_cleanup() {
    int t = -1;
    const int st_timing = jpge_set_timing(g_ctx, 1);           // released: JPGE_E_ARG
    const int st_lanes = jpge_get_lanes(g_ctx, &t);             // released: JPGE_E_ARG
    const int st_close = jpge_close(g_ctx);                     // no-op
    const int st_close2 = jpge_close(g_ctx);                    // still a no-op
    const int st_gsize = jpge_group_size(g_grp, &t, nullptr);   // released: JPGE_E_ARG
    const int st_gclose = jpge_group_close(g_grp);              // no-op
    if (st_timing == JPGE_E_ARG && st_lanes == JPGE_E_ARG && st_close == JPGE_OK && st_close2 == JPGE_OK &&
        st_gsize == JPGE_E_ARG && st_gclose == JPGE_OK)
        std::printf("cleanup ok\n");
    else
        std::printf("cleanup FAILED %d %d %d %d %d %d\n", st_timing, st_lanes, st_close, st_close2, st_gsize,
                    st_gclose);
    std::fflush(stdout);
}

int main() {
    std::atexit(caller_cleanup);  // before jpge_open: runs AFTER the library's handler
    if (jpge_open(0, &g_ctx) != JPGE_OK) return 2;
    const int dev[2] = {0, 0};
    if (jpge_group_open(2, dev, 1, &g_grp) != JPGE_OK) return 3;
    const uint32_t w = 96, h = 64;
    std::vector<uint8_t> rgb(w * h * 3);
    for (size_t i = 0; i < rgb.size(); ++i) rgb[i] = (uint8_t)(i * 7 + (i >> 5));
    uint8_t qy[64], qc[64];
    jpge_quality_tables(90, qy, qc);
    std::vector<uint8_t> out(jpge_max_jpeg_bytes(w, h));
    size_t len = 0;
    if (jpge_encode_rgb8(g_ctx, rgb.data(), w, h, w * 3, 255, qy, qc, out.data(), out.size(), &len, 0) != JPGE_OK)
        return 4;
    std::printf("encoded %zu bytes\n", len);
    return 0;  // exit(): the library's handler, then caller_cleanup
}
