// Diagnostic: host threads' CPU while the GPU is busy, per HIP usage pattern (each
// phase keeps a stream busy ~0.5 s with short kernels and prints threads above 5%).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <dirent.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <thread>

static std::map<std::string, double> cpu() {
    std::map<std::string, double> m;
    DIR* d = opendir("/proc/self/task");
    while (dirent* e = readdir(d)) {
        if (e->d_name[0] == '.') continue;
        char p[256], b[1024];
        snprintf(p, sizeof p, "/proc/self/task/%s/stat", e->d_name);
        FILE* f = fopen(p, "r");
        if (!f) continue;
        size_t n = fread(b, 1, sizeof b - 1, f);
        fclose(f);
        b[n] = 0;
        char* r = strrchr(b, ')');
        long ut = 0, st = 0;
        sscanf(r + 2, "%*c %*d %*d %*d %*d %*d %*u %*u %*u %*u %*u %ld %ld", &ut, &st);
        m[e->d_name] = (ut + st) / (double)sysconf(_SC_CLK_TCK);
    }
    closedir(d);
    return m;
}
__global__ void spin(int* p, long long n) {
    long long t0 = clock64();
    while (clock64() - t0 < n) {}
    if (threadIdx.x == 0) p[blockIdx.x] = 1;
}
template <class F>
static void phase(const char* what, F&& f) {
    auto a = cpu();
    auto t0 = std::chrono::steady_clock::now();
    f();
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    auto b = cpu();
    printf("%-44s %.2fs", what, dt);
    for (auto& kv : b) {
        double u = (kv.second - a[kv.first]) / dt;
        if (u > 0.05) printf(" %s:%.2f", kv.first.c_str(), u);
    }
    printf("  (%zu threads)\n", b.size());
}
int main() {
    hipSetDevice(0);
    int* d;
    hipMalloc(&d, 1 << 20);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const long long cyc = 20000;  // ~10 us kernels
    phase("5000 kernels, stream sync at the end", [&] {
        for (int i = 0; i < 5000; ++i) hipLaunchKernelGGL(spin, dim3(256), dim3(64), 0, s, d, cyc);
        hipStreamSynchronize(s);
    });
    phase("5000 kernels, spin on hipEventQuery", [&] {
        for (int i = 0; i < 5000; ++i) hipLaunchKernelGGL(spin, dim3(256), dim3(64), 0, s, d, cyc);
        hipEventRecord(e0, s);
        while (hipEventQuery(e0) == hipErrorNotReady) {}
    });
    phase("5000 kernels + event record each", [&] {
        for (int i = 0; i < 5000; ++i) {
            hipLaunchKernelGGL(spin, dim3(256), dim3(64), 0, s, d, cyc);
            hipEventRecord(e0, s);
        }
        hipStreamSynchronize(s);
    });
    phase("5000 kernels via hipExtLaunchKernel events", [&] {
        for (int i = 0; i < 5000; ++i) hipExtLaunchKernelGGL(spin, dim3(256), dim3(64), 0, s, e0, e1, 0, d, cyc);
        hipStreamSynchronize(s);
    });
    phase("idle 0.3 s after", [&] { std::this_thread::sleep_for(std::chrono::milliseconds(300)); });
    void* h;
    hipHostMalloc(&h, 4096, hipHostMallocMapped);
    phase("5000 kernels, mapped host memory", [&] {
        for (int i = 0; i < 5000; ++i) hipLaunchKernelGGL(spin, dim3(256), dim3(64), 0, s, (int*)h, cyc);
        hipStreamSynchronize(s);
    });
    return 0;
}
