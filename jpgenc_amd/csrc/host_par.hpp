// Spawn-and-join parallel loop for the host side.  Threads end with the call, so
// nothing is left polling afterwards: an OpenMP runtime keeps its team spinning
// for its block time (LLVM libomp: 200 ms), which on a CPU-quota'd host starves
// the encoder's pipeline threads.
#pragma once
#include <algorithm>
#include <thread>
#include <vector>

namespace jpge {

// fn(i) for i in [0, n), split into `threads` contiguous ranges (the caller runs one).
template <class F>
void parallel_for(long n, int threads, F&& fn) {
    threads = (int)std::max(1L, std::min<long>(threads, n));
    if (threads == 1) {
        for (long i = 0; i < n; ++i) fn(i);
        return;
    }
    std::vector<std::thread> th;
    th.reserve(threads - 1);
    auto range = [&](int t) {
        const long lo = n * t / threads, hi = n * (t + 1) / threads;
        for (long i = lo; i < hi; ++i) fn(i);
    };
    for (int t = 1; t < threads; ++t) th.emplace_back(range, t);
    range(0);
    for (auto& x : th) x.join();
}

}  // namespace jpge
