// Diagnostic: host CPU per operation of a lane thread's loop, on the GPU box (thread
// CPU time from CLOCK_THREAD_CPUTIME_ID): kernel launches (plain and with events bound
// to the dispatch), 10 us naps, mapped-memory polls.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <sys/prctl.h>
#include <time.h>
#include <chrono>
#include <cstdio>
#include <thread>

__global__ void empty_kernel(int* p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 1;
}

static double tcpu_us() {
    timespec t;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}
static double wall_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    int* d;
    hipMalloc(&d, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int N = 20000;
    for (int i = 0; i < 1000; ++i) hipLaunchKernelGGL(empty_kernel, dim3(512), dim3(256), 0, s, d);
    hipStreamSynchronize(s);
    {
        double c0 = tcpu_us(), w0 = wall_us();
        for (int i = 0; i < N; ++i) {
            hipLaunchKernelGGL(empty_kernel, dim3(512), dim3(256), 0, s, d);
            if ((i & 255) == 255) hipStreamSynchronize(s);
        }
        hipStreamSynchronize(s);
        printf("hipLaunchKernelGGL: %.2f us CPU, %.2f us wall per launch\n", (tcpu_us() - c0) / N, (wall_us() - w0) / N);
    }
    {
        double c0 = tcpu_us(), w0 = wall_us();
        for (int i = 0; i < N; ++i) {
            hipExtLaunchKernelGGL(empty_kernel, dim3(512), dim3(256), 0, s, e0, e1, 0, d);
            if ((i & 255) == 255) hipStreamSynchronize(s);
        }
        hipStreamSynchronize(s);
        printf("hipExtLaunchKernelGGL with events: %.2f us CPU, %.2f us wall per launch\n", (tcpu_us() - c0) / N,
               (wall_us() - w0) / N);
    }
    for (unsigned long slack : {50000UL, 1000UL}) {
        prctl(PR_SET_TIMERSLACK, slack, 0, 0, 0);
        const int M = 20000;
        double c0 = tcpu_us(), w0 = wall_us();
        for (int i = 0; i < M; ++i) std::this_thread::sleep_for(std::chrono::microseconds(10));
        printf("sleep_for(10us), slack %lu ns: %.2f us CPU, %.2f us wall per call\n", slack, (tcpu_us() - c0) / M,
               (wall_us() - w0) / M);
    }
    {
        const int M = 2000;
        double c0 = tcpu_us(), w0 = wall_us();
        for (int i = 0; i < M; ++i) std::this_thread::sleep_for(std::chrono::microseconds(100));
        printf("sleep_for(100us): %.2f us CPU, %.2f us wall per call\n", (tcpu_us() - c0) / M, (wall_us() - w0) / M);
    }
    return 0;
}
