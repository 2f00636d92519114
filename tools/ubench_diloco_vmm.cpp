// r04 experiment: physical chunks (HIP virtual memory management) as placement
// candidates for the fused DiLoCo step (ga_diloco_outer, K = 8, GPT-2 124M).
// (1) 48 physical chunks of 1 GiB (hipMemCreate, one at a time), mapped at
//     consecutive 1 GiB slots of one reserved VA range; the replica set a plain
//     hipMalloc (as the product allocates it); each chunk timed as master+momentum
//     (0.5 + 0.5 GiB) -> a fast/slow map of the chunks against these replicas.
// (2) replica sets built from chunks: four chunks (1 GiB each) from the slow class,
//     two slow + two fast, and alternating; master+momentum in a chunk of a class.
// Not part of the library.
//   hipcc -O2 --offload-arch=gfx950 tools/ubench_diloco_vmm.cpp -Lgym_amd/_lib -lgym_amd \
//         -Wl,-rpath,'$ORIGIN/../gym_amd/_lib' -o build/ubench_diloco_vmm
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../include/gym_amd.h"

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

static const int64_t K = 8;
static const int64_t N = 124475904;

static float run(float* rep, int64_t ld, float* master, float* mom, int reps, hipStream_t s) {
    auto launch = [&] {
        if (ga_diloco_outer(GA_F32, rep, K, ld, N, (float)K, master, mom, 1, 0, 0.7f, 0.9f, 0.f, 0.f, 1, rep, K, ld,
                            s)) {
            printf("ga_diloco_outer: %s\n", ga_last_error());
            exit(1);
        }
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch();
    CK(hipStreamSynchronize(s));
    float best = 1e9f;
    for (int r = 0; r < 2; ++r) {
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms / reps < best) best = ms / reps;
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return best;
}

// (3) the replica set itself as K row chunks mapped into one VA range, with `spacer` GiB of
// held physical memory created between consecutive rows (released after), then master+mom
// probed over 24 candidates: best and median step time per spacer size
static void rows_spread(hipStream_t s, const hipMemAllocationProp& prop, const hipMemAccessDesc& acc) {
    const int64_t G1 = 1LL << 30;
    const int64_t ld = (N + 1023) / 1024 * 1024;  // rows a multiple of 4 KiB
    const int64_t row_b = 4 * ld;
    for (int spacer : {0, 2, 4, 8}) {
        void* va = nullptr;
        CK(hipMemAddressReserve(&va, (size_t)(K * row_b), 2 << 20, nullptr, 0));
        std::vector<hipMemGenericAllocationHandle_t> rows(K), sp;
        for (int k = 0; k < K; ++k) {
            CK(hipMemCreate(&rows[k], row_b, (hipMemAllocationProp*)&prop, 0));
            CK(hipMemMap((char*)va + k * row_b, row_b, 0, rows[k], 0));
            for (int j = 0; j < spacer && k + 1 < K; ++j) {
                hipMemGenericAllocationHandle_t h;
                CK(hipMemCreate(&h, G1, (hipMemAllocationProp*)&prop, 0));
                sp.push_back(h);
            }
        }
        CK(hipMemSetAccess(va, (size_t)(K * row_b), &acc, 1));
        CK(hipMemset(va, 0, (size_t)(K * row_b)));
        for (auto h : sp) CK(hipMemRelease(h));
        std::vector<float> ts;
        std::vector<std::pair<void*, hipMemGenericAllocationHandle_t>> cands;
        for (int c = 0; c < 24; ++c) {
            hipMemGenericAllocationHandle_t h;
            void* cv = nullptr;
            CK(hipMemCreate(&h, G1, (hipMemAllocationProp*)&prop, 0));
            CK(hipMemAddressReserve(&cv, G1, 2 << 20, nullptr, 0));
            CK(hipMemMap(cv, G1, 0, h, 0));
            CK(hipMemSetAccess(cv, G1, &acc, 1));
            cands.push_back({cv, h});
            ts.push_back(run((float*)va, ld, (float*)cv, (float*)cv + N, 5, s));
        }
        std::vector<float> st = ts;
        std::sort(st.begin(), st.end());
        printf("(3) rows as chunks, %d GiB spacers: master+mom best %.3f median %.3f worst %.3f ms | ", spacer, st[0],
               st[st.size() / 2], st.back());
        for (float x : ts) printf("%.2f ", x);
        printf("\n");
        fflush(stdout);
        for (auto& c : cands) {
            CK(hipMemUnmap(c.first, G1));
            CK(hipMemAddressFree(c.first, G1));
            CK(hipMemRelease(c.second));
        }
        CK(hipMemUnmap(va, (size_t)(K * row_b)));
        CK(hipMemAddressFree(va, (size_t)(K * row_b)));
        for (auto h : rows) CK(hipMemRelease(h));
    }
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int dev = 0, vmm = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, dev));
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    size_t gran = 0;
    CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    printf("VMM supported %d, granularity %zu B\n", vmm, gran);
    if (getenv("ROWS_SPREAD")) {
        hipMemAccessDesc acc0 = {};
        acc0.location = prop.location;
        acc0.flags = hipMemAccessFlagsProtReadWrite;
        rows_spread(s, prop, acc0);
        return 0;
    }
    const int64_t G1 = 1LL << 30;
    const int nch = 48;
    void* va = nullptr;
    CK(hipMemAddressReserve(&va, (size_t)nch * G1, G1, nullptr, 0));
    std::vector<hipMemGenericAllocationHandle_t> h(nch);
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    for (int i = 0; i < nch; ++i) {
        CK(hipMemCreate(&h[i], G1, &prop, 0));
        CK(hipMemMap((char*)va + i * G1, G1, 0, h[i], 0));
    }
    CK(hipMemSetAccess(va, (size_t)nch * G1, &acc, 1));
    CK(hipMemset(va, 0, (size_t)nch * G1));
    float* rep;
    CK(hipMalloc(&rep, 4 * K * N));
    CK(hipMemset(rep, 0, 4 * K * N));
    auto chunk = [&](int i) { return (float*)((char*)va + i * G1); };
    std::vector<float> t(nch);
    printf("(1) master+mom in chunk i against a hipMalloc'd replica set:\n");
    for (int i = 0; i < nch; ++i) {
        t[i] = run(rep, N, chunk(i), chunk(i) + N, 5, s);
        printf("  %2d %.3f%s", i, t[i], i % 8 == 7 ? "\n" : "");
    }
    // classes by time: fast < midpoint
    float lo = 1e9f, hi = 0.f;
    for (float x : t) { lo = x < lo ? x : lo; hi = x > hi ? x : hi; }
    const float mid = 0.5f * (lo + hi);
    std::vector<int> fast, slow;
    for (int i = 0; i < nch; ++i) (t[i] < mid ? fast : slow).push_back(i);
    printf("fast %zu slow %zu (split at %.3f)\n", fast.size(), slow.size(), mid);
    // (2) replica sets from chunks: a second reserved range of 4 GiB + master/mom 1 GiB
    if (fast.size() >= 6 && slow.size() >= 6) {
        void* va2 = nullptr;
        const int64_t rows_b = 4 * K * N;  // 3.98 GB -> 4 chunks
        CK(hipMemAddressReserve(&va2, 5 * G1, G1, nullptr, 0));
        auto build = [&](std::vector<int> cs, int mm) {
            for (int j = 0; j < 4; ++j) CK(hipMemMap((char*)va2 + j * G1, G1, 0, h[cs[j]], 0));
            CK(hipMemMap((char*)va2 + 4 * G1, G1, 0, h[mm], 0));
            CK(hipMemSetAccess(va2, 5 * G1, &acc, 1));
            const float tt = run((float*)va2, N, (float*)((char*)va2 + 4 * G1), (float*)((char*)va2 + 4 * G1) + N, 5, s);
            CK(hipMemUnmap(va2, 5 * G1));
            return tt;
        };
        (void)rows_b;
        struct V { const char* name; std::vector<int> cs; int mm; };
        std::vector<V> vs = {
            {"rows slow x4, mm slow", {slow[0], slow[1], slow[2], slow[3]}, slow[4]},
            {"rows slow x4, mm fast", {slow[0], slow[1], slow[2], slow[3]}, fast[4]},
            {"rows fast x4, mm fast", {fast[0], fast[1], fast[2], fast[3]}, fast[4]},
            {"rows fast x4, mm slow", {fast[0], fast[1], fast[2], fast[3]}, slow[4]},
            {"rows s,f,s,f, mm slow", {slow[0], fast[0], slow[1], fast[1]}, slow[4]},
            {"rows s,f,s,f, mm fast", {slow[0], fast[0], slow[1], fast[1]}, fast[4]},
            {"rows s,s,f,f, mm fast", {slow[0], slow[1], fast[0], fast[1]}, fast[4]},
            {"rows spread chunks, mm", {slow[0], slow[slow.size() / 2], fast[0], fast[fast.size() / 2]}, fast.back()},
        };
        printf("(2) replica set (4 x 1 GiB chunks) + master/mom chunk:\n");
        for (int r = 0; r < 2; ++r)
            for (auto& v : vs) printf("  %-26s %.3f ms\n", v.name, build(v.cs, v.mm));
    }
    return 0;
}
