// Diagnostic: which HIP runtime calls leave a host thread spinning?  Each phase
// runs, then the process idles 0.5 s and prints every thread's CPU time in that
// window (from /proc/self/task).
#include <hip/hip_runtime.h>
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
static void idle(const char* what) {
    auto a = cpu();
    std::this_thread::sleep_for(std::chrono::milliseconds(500));
    auto b = cpu();
    printf("%-40s", what);
    for (auto& kv : b) {
        double u = (kv.second - a[kv.first]) / 0.5;
        if (u > 0.05) printf(" %s:%.2f", kv.first.c_str(), u);
    }
    printf("  (%zu threads)\n", b.size());
}
__global__ void k(int* p) { p[threadIdx.x] += 1; }
int main() {
    idle("start");
    int n;
    hipGetDeviceCount(&n);
    idle("hipGetDeviceCount");
    hipSetDevice(0);
    int* d;
    hipMalloc(&d, 4096);
    idle("hipMalloc");
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    idle("stream");
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, s, d);
    hipStreamSynchronize(s);
    idle("kernel+sync");
    void* h;
    hipHostMalloc(&h, 4096, hipHostMallocMapped);
    idle("hipHostMalloc mapped");
    hipEvent_t e;
    hipEventCreate(&e);
    hipEventRecord(e, s);
    while (hipEventQuery(e) == hipErrorNotReady) {}
    idle("event record+query");
    for (int i = 0; i < 1000; ++i) hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, s, d);
    hipStreamSynchronize(s);
    idle("1000 kernels");
    return 0;
}
