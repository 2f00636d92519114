// Does the ORDER of the replica-mode SPARTA step's random words matter?  The rows
// layout [K, ld] (K = 32 replicas of GPT-2 124M, fp32) and M = 0.005 n sorted
// selected positions: every (position, replica) word is read and written once.
//   element-major: consecutive threads take the K replicas of one position (what the
//                  rows kernel does: one lane per element, its K words back to back)
//   replica-major: consecutive threads take consecutive positions of one replica row
//                  (a row's words in ascending address order)
// Read-modify-write (x += 1), read-only (sum), write-only variants.  Standalone
// diagnostic (round 5).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <random>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int MODE, bool EM>  // MODE 0 rmw, 1 read, 2 write
__global__ void words(float* __restrict__ rows, long ld, const int* __restrict__ pos, int M, int K, float* sink) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)M * K) return;
    int e, k;
    if (EM) { e = (int)(i / K); k = (int)(i - (long)e * K); }
    else { k = (int)(i / M); e = (int)(i - (long)k * M); }
    float* a = rows + (long)k * ld + pos[e];
    if (MODE == 0) *a += 1.f;
    else if (MODE == 1) { const float v = *a; if (v == 1234.5f) sink[0] = v; }
    else *a = (float)k;
}

template <typename F>
float time_ms(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    const long n = 124475904L, ld = n;
    const int K = 32;
    const int M = (int)(n * 0.005);
    std::vector<int> hp(M);
    std::mt19937_64 g(5);
    std::uniform_int_distribution<long> u(0, n - 1);
    for (int i = 0; i < M; ++i) hp[i] = (int)u(g);
    std::sort(hp.begin(), hp.end());
    float *rows, *sink;
    int* pos;
    CK(hipMalloc(&rows, sizeof(float) * ld * K));
    CK(hipMalloc(&pos, sizeof(int) * M));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(rows, 0, sizeof(float) * ld * K));
    CK(hipMemcpy(pos, hp.data(), sizeof(int) * M, hipMemcpyHostToDevice));
    const long tot = (long)M * K;
    const int blk = 256;
    const int grid = (int)((tot + blk - 1) / blk);
#define RUN(MODE, EM, what) for (int r = 0; r < 3; ++r) { float ms = time_ms([&] { words<MODE, EM><<<grid, blk>>>(rows, ld, pos, M, K, sink); }, 10); \
        printf("%-14s %-6s %.3f ms  (%ld words)\n", EM ? "element-major" : "replica-major", what, ms, tot); }
    RUN(0, true, "rmw") RUN(0, false, "rmw")
    RUN(1, true, "read") RUN(1, false, "read")
    RUN(2, true, "write") RUN(2, false, "write")
    return 0;
}
