// r04 layout experiment for ga_diloco_outer (K = 8, GPT-2 124M, fp32): the library
// kernel through the C ABI, timed under controlled placements of its 10 streams, all
// interleaved in ONE process (rounds x layouts), so layout effects and between-process
// effects can be told apart.  Not part of the library.
//   hipcc -O2 --offload-arch=gfx950 tools/ubench_diloco_layout.cpp -Lgym_amd/_lib -lgym_amd \
//         -Wl,-rpath,'$ORIGIN/../gym_amd/_lib' -o build/ubench_diloco_layout
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
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
static const int64_t N = 124475904;  // GPT-2 124M arena
static const int64_t MiB2 = 2 << 20;

struct Layout {
    std::string name;
    float* rep;    // replica 0
    int64_t ld;    // replica stride (elements)
    float* master;
    float* mom;
};

static int64_t up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

static float run(const Layout& L, int reps, hipStream_t s) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto launch = [&] {
        int rc = ga_diloco_outer(GA_F32, L.rep, K, L.ld, N, (float)K, L.master, L.mom, 1, 0, 0.7f, 0.9f,
                                 0.f, 0.f, 1, L.rep, K, L.ld, s);
        if (rc) {
            printf("ga_diloco_outer: %s\n", ga_last_error());
            exit(1);
        }
    };
    launch();
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms / reps;
}

static float run_copy(float* a, float* b, int64_t bytes, int reps, hipStream_t s) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    ga_stream_copy(a, b, bytes, s);
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i) ga_stream_copy(a, b, bytes, s);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

static void describe(const Layout& L) {
    const uintptr_t p[3] = {(uintptr_t)L.rep, (uintptr_t)L.master, (uintptr_t)L.mom};
    printf("# %-14s ld=%lld (stride %% 2MiB = %lld B) rep0%%2M=%llu rep0%%256M=%llu master%%2M=%llu "
           "master%%256M=%llu mom%%2M=%llu mom%%256M=%llu\n",
           L.name.c_str(), (long long)L.ld, (long long)((L.ld * 4) % MiB2),
           (unsigned long long)(p[0] % MiB2), (unsigned long long)(p[0] % (256 << 20)),
           (unsigned long long)(p[1] % MiB2), (unsigned long long)(p[1] % (256 << 20)),
           (unsigned long long)(p[2] % MiB2), (unsigned long long)(p[2] % (256 << 20)));
}

// search mode: replicas packed at the start of a pool, master and momentum at
// pseudo-random 64 KiB-aligned offsets past them (the same offsets in every process
// for one seed); each placement timed twice, then the 6 fastest re-timed 3 times
static int search(int seed, int ncand, int reps, hipStream_t s) {
    const int64_t pool_bytes = (int64_t)24 << 30;
    char* pool;
    CK(hipMalloc(&pool, pool_bytes));
    CK(hipMemset(pool, 0, pool_bytes));
    const int64_t rows_b = 4 * K * N, one_b = 4 * N, gran = 64 << 10;
    const int64_t span = (pool_bytes - rows_b - 2 * one_b) / gran;
    uint64_t st = 0x9E3779B97F4A7C15ull * (uint64_t)(seed + 1);
    auto rnd = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; };
    struct C { int64_t a, b; float t; };
    std::vector<C> cs;
    while ((int)cs.size() < ncand) {
        int64_t a = rows_b + (int64_t)(rnd() % span) * gran, b = rows_b + (int64_t)(rnd() % span) * gran;
        if ((a < b ? b - a : a - b) < one_b) continue;  // master and momentum must not overlap
        cs.push_back({a, b, 0.f});
    }
    auto lay = [&](const C& c) { return Layout{"cand", (float*)pool, N, (float*)(pool + c.a), (float*)(pool + c.b)}; };
    const double alg = (2.0 * K + 4.0) * 4.0 * N;
    for (auto& c : cs) {
        const float t0 = run(lay(c), reps, s), t1 = run(lay(c), reps, s);
        c.t = t0 < t1 ? t0 : t1;
        printf("cand master@%lld (%%2M %lld, %%1G %lld) mom@%lld (%%2M %lld) d=%lld: %.4f %.4f ms frac %.3f\n",
               (long long)c.a, (long long)(c.a % MiB2), (long long)(c.a % (1LL << 30)), (long long)c.b,
               (long long)(c.b % MiB2), (long long)(c.b - c.a), t0, t1, alg / c.t / 1e6 / 8000.0);
    }
    std::vector<C> srt = cs;
    for (size_t i = 0; i < srt.size(); ++i)
        for (size_t j = i + 1; j < srt.size(); ++j)
            if (srt[j].t < srt[i].t) std::swap(srt[i], srt[j]);
    for (int r = 0; r < 3; ++r)
        for (int i = 0; i < 6 && i < (int)srt.size(); ++i) {
            const float t = run(lay(srt[i]), reps, s);
            printf("best%d r%d master@%lld mom@%lld: %.4f ms frac %.3f\n", i, r, (long long)srt[i].a,
                   (long long)srt[i].b, t, alg / t / 1e6 / 8000.0);
        }
    const int w = (int)srt.size() - 1;
    printf("worst master@%lld mom@%lld: %.4f ms\n", (long long)srt[w].a, (long long)srt[w].b, srt[w].t);
    return 0;
}

// sweep mode: one 60 GiB pool; (a) replicas packed at 0, master + momentum adjacent at
// 1 GiB steps from 4 to 52 GiB; (b) replicas packed at 16 / 32 GiB with master +
// momentum at 0; (c) replica rows spread S GiB apart with master + momentum after them
static int sweep(int reps, hipStream_t s) {
    const int64_t G1 = 1LL << 30;
    const int64_t pool_bytes = 60 * G1;
    char* pool;
    CK(hipMalloc(&pool, pool_bytes));
    CK(hipMemset(pool, 0, pool_bytes));
    const double alg = (2.0 * K + 4.0) * 4.0 * N;
    auto time2 = [&](const Layout& L) { const float a = run(L, reps, s), b = run(L, reps, s); return a < b ? a : b; };
    auto at = [&](int64_t off) { return (float*)(pool + off); };
    const int64_t one_b = 4 * N;
    for (int64_t g = 4; g <= 52; ++g) {
        const Layout L{"a", at(0), N, at(g * G1), at(g * G1 + one_b)};
        const float t = time2(L);
        printf("a replicas@0 master@%lldG mom adjacent: %.4f ms frac %.3f\n", (long long)g, t, alg / t / 1e6 / 8000.0);
    }
    for (int64_t r : {16LL, 32LL, 48LL}) {
        const Layout L{"b", at(r * G1), N, at(0), at(one_b)};
        const float t = time2(L);
        printf("b replicas@%lldG master@0 mom adjacent: %.4f ms frac %.3f\n", (long long)r, t, alg / t / 1e6 / 8000.0);
    }
    for (int64_t S : {1LL, 2LL, 4LL, 6LL}) {
        const int64_t ld = S * G1 / 4;
        const Layout L{"c", at(0), ld, at(K * S * G1), at(K * S * G1 + one_b)};
        if (K * S * G1 + 2 * one_b > pool_bytes) continue;
        const float t = time2(L);
        printf("c rows %lldG apart, master@%lldG: %.4f ms frac %.3f\n", (long long)S, (long long)(K * S), t,
               alg / t / 1e6 / 8000.0);
    }
    fflush(stdout);
    return 0;
}

// map mode: a 100 GiB pool; (A) the replica set in its own allocation (as the product
// allocates it), master + momentum adjacent at 2 GiB steps over the pool; (B) the
// replica set at pool offset R (8 GiB steps), master + momentum at pool offset M
// (8 GiB steps): the (R, M) grid of step times
static int map_mode(int reps, hipStream_t s) {
    const int64_t G1 = 1LL << 30;
    const int64_t pool_bytes = 100 * G1;
    const int64_t one_b = 4 * N, rows_b = 4 * K * N;
    float* rep;
    CK(hipMalloc(&rep, rows_b));
    CK(hipMemset(rep, 0, rows_b));
    char* pool;
    CK(hipMalloc(&pool, pool_bytes));
    CK(hipMemset(pool, 0, pool_bytes));
    auto at = [&](int64_t off) { return (float*)(pool + off); };
    auto t1 = [&](const Layout& L) { const float a = run(L, reps, s), b = run(L, reps, s); return a < b ? a : b; };
    printf("A (replicas in their own allocation; master+mom at pool offset g GiB):\n");
    for (int64_t g = 0; g + 1 < 100; g += 2) {
        const float t = t1(Layout{"a", rep, N, at(g * G1), at(g * G1 + one_b)});
        printf("  g=%3lld %.3f%s", (long long)g, t, (g / 2) % 8 == 7 ? "\n" : "");
    }
    printf("\nB (replicas at pool offset R GiB, master+mom at pool offset M GiB), ms:\n      ");
    for (int64_t M = 0; M < 100; M += 8) printf(" M=%-4lld", (long long)M);
    printf("\n");
    for (int64_t R = 0; R + 4 < 100; R += 8) {
        printf("R=%3lld", (long long)R);
        for (int64_t M = 0; M < 100; M += 8) {
            if (M + 1 > R && M < R + 5) {
                printf("   --  ");
                continue;
            }
            printf(" %.3f", t1(Layout{"b", at(R * G1), N, at(M * G1), at(M * G1 + one_b)}));
        }
        printf("\n");
        fflush(stdout);
    }
    return 0;
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 4;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    if (argc > 3 && !strcmp(argv[3], "sweep")) return sweep(reps, s);
    if (argc > 3 && !strcmp(argv[3], "map")) return map_mode(reps, s);
    if (argc > 3 && !strcmp(argv[3], "search")) return search(argc > 4 ? atoi(argv[4]) : 0, argc > 5 ? atoi(argv[5]) : 40, reps, s);
    std::vector<Layout> Ls;
    // (a) the product's allocation: replica set, master, momentum as separate allocations
    // (torch.empty of [K, n], then DiLoCoOuter's two buffers)
    float *rep_a, *m_a, *b_a;
    CK(hipMalloc(&rep_a, 4 * K * N));
    CK(hipMalloc(&m_a, 4 * N));
    CK(hipMalloc(&b_a, 4 * N));
    Ls.push_back({"separate", rep_a, N, m_a, b_a});
    // (b) one pool; the other layouts are placements inside it
    const int64_t ld2m = up(N * 4, MiB2) / 4;  // row stride a whole number of 2 MiB pages
    const int64_t pool_bytes = (int64_t)14 << 30;
    char* pool;
    CK(hipMalloc(&pool, pool_bytes));
    CK(hipMemset(pool, 0, pool_bytes));
    auto at = [&](int64_t off) { return (float*)(pool + off); };
    const int64_t rows_b = 4 * K * N, one_b = 4 * N;
    Ls.push_back({"pool-packed", at(0), N, at(rows_b), at(rows_b + one_b)});
    Ls.push_back({"pool-2M", at(0), ld2m, at(K * ld2m * 4), at(K * ld2m * 4 + up(one_b, MiB2))});
    for (int64_t st : {(int64_t)4096, (int64_t)65536, (int64_t)262144, (int64_t)(MiB2 / 8 * 3)}) {
        // row k offset by k * st within the 2 MiB page: rows land on different channel phases
        const int64_t ld = ld2m + st / 4;
        const int64_t m_off = up(K * ld * 4, MiB2) + K * st;
        Ls.push_back({"pool-stag" + std::to_string(st / 1024) + "k", at(0), ld, at(m_off),
                      at(m_off + up(one_b, MiB2) + (K + 1) * st)});
    }
    Ls.push_back({"pool-mm-first", at(2 * up(one_b, MiB2)), N, at(0), at(up(one_b, MiB2))});
    Ls.push_back({"pool-off1G", at((int64_t)1 << 30), N, at((1LL << 30) + rows_b), at((1LL << 30) + rows_b + one_b)});
    Ls.push_back({"pool-off7G", at((int64_t)7 << 30), N, at((7LL << 30) + rows_b), at((7LL << 30) + rows_b + one_b)});
    CK(hipMemset(rep_a, 0, 4 * K * N));
    CK(hipMemset(m_a, 0, 4 * N));
    CK(hipMemset(b_a, 0, 4 * N));
    for (auto& L : Ls) describe(L);
    float* cbuf;
    CK(hipMalloc(&cbuf, (int64_t)5 << 30));
    const int64_t cbytes = (int64_t)2400 << 20;  // ~ half the DiLoCo stream each way
    const double alg = (2.0 * K + 4.0) * 4.0 * N;
    for (int r = 0; r < rounds; ++r) {
        const float cm = run_copy((float*)cbuf, (float*)(cbuf + cbytes), cbytes, reps, s);
        printf("round %d copy %.4f ms %.0f GB/s\n", r, cm, 2.0 * cbytes / cm / 1e6);
        for (auto& L : Ls) {
            const float ms = run(L, reps, s);
            printf("round %d %-14s %.4f ms %.0f GB/s frac %.3f\n", r, L.name.c_str(), ms, alg / ms / 1e6,
                   alg / ms / 1e6 / 8000.0);
        }
        fflush(stdout);
    }
    return 0;
}
