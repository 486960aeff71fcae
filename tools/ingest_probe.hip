// Development probe (not part of the library): how fast can a k_ingest-shaped grid load its
// columns?  1024 chunks x 512 threads x RPT rows, three int64 columns (CFG2's key / ts / value),
// with optional per-row arithmetic standing in for the murmur + key-group + slice-end work.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/ingest_probe tools/ingest_probe.hip && /tmp/ingest_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#include "../flink_amd/csrc/fw_internal.h"

using namespace fw;

constexpr int NB = 32;

template <int BLOCK, int RPT, int WORK>
__global__ __launch_bounds__(BLOCK) void k_probe(const int64_t* __restrict__ key, const int64_t* __restrict__ ts,
                                                 const int64_t* __restrict__ val, int64_t* out) {
    const int64_t base = (int64_t)blockIdx.x * BLOCK * RPT;
    int64_t rk[RPT], rs[RPT], rv[RPT];
#pragma unroll
    for (int j = 0; j < RPT; j++) {
        const int64_t o = base + j * BLOCK + threadIdx.x;
        rk[j] = key[o];
        rs[j] = ts[o];
        rv[j] = val[o];
    }
    uint64_t acc = 0;
#pragma unroll
    for (int j = 0; j < RPT; j++) {
        uint32_t h = (uint32_t)rk[j] ^ (uint32_t)(rk[j] >> 32);
#pragma unroll
        for (int w = 0; w < WORK; w++) {  // murmur-like mixing rounds
            h *= 0xcc9e2d51u;
            h = (h << 15) | (h >> 17);
            h *= 0x1b873593u;
            h ^= h >> 13;
        }
        const uint64_t se = (uint64_t)rs[j] / 10000u;
        acc += h + se + (uint64_t)rv[j];
    }
    __shared__ uint64_t red[BLOCK / 64];
#pragma unroll
    for (int k = 32; k > 0; k >>= 1) acc += __shfl_xor(acc, k, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t s = 0;
        for (int i = 0; i < BLOCK / 64; i++) s += red[i];
        out[blockIdx.x] = (int64_t)s;
    }
}

// the ingest's own per-row routing and slice arithmetic (route_key with BinaryRowData BIGINT keys,
// 32-bit slice end), optionally counting rows per superbucket in an LDS histogram
template <int BLOCK, int RPT, int HIST>
__global__ __launch_bounds__(BLOCK) void k_real(const int64_t* __restrict__ key, const int64_t* __restrict__ ts,
                                                const int64_t* __restrict__ val, int64_t* out, KeySpace ks,
                                                UDiv32 sdiv, int64_t interval) {
    __shared__ uint32_t hist[1024];
    __shared__ uint64_t red[BLOCK / 64];
    for (int i = threadIdx.x; i < 1024; i += BLOCK) hist[i] = 0;
    const int64_t base = (int64_t)blockIdx.x * BLOCK * RPT;
    int64_t rk[RPT], rs[RPT], rv[RPT];
#pragma unroll
    for (int j = 0; j < RPT; j++) {
        const int64_t o = base + j * BLOCK + threadIdx.x;
        rk[j] = key[o];
        rs[j] = ts[o];
        rv[j] = val[o];
    }
    const int64_t tbase = ts[base] - (1 << 29);
    __syncthreads();
    uint64_t acc = 0;
    int64_t lmin = INT64_MAX;
#pragma unroll
    for (int j = 0; j < RPT; j++) {
        uint32_t m;
        const int32_t sb = route_key(ks, rk[j], 0, &m, KH_BINROW_BIGINT);
        const uint32_t d32 = (uint32_t)(rs[j] - tbase);
        const uint32_t r = d32 - udiv32(d32, sdiv) * (uint32_t)interval;
        const int64_t se = rs[j] - (int64_t)r + interval;
        lmin = min(lmin, se);
        if (HIST) atomicAdd(&hist[sb & 1023], 1u);
        acc += (uint64_t)sb + (uint64_t)rv[j];
    }
    __syncthreads();
    if (HIST) acc += hist[threadIdx.x & 1023];
    acc += (uint64_t)lmin;
#pragma unroll
    for (int k = 32; k > 0; k >>= 1) acc += __shfl_xor(acc, k, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t s = 0;
        for (int i = 0; i < BLOCK / 64; i++) s += red[i];
        out[blockIdx.x] = (int64_t)s;
    }
}

template <int BLOCK, int RPT, int HIST>
static void run_real(const char* name, const int64_t* k0, const int64_t* t0, const int64_t* v0, int64_t* out, int64_t n) {
    const int grid = (int)(n / (BLOCK * RPT));
    KeySpace ks{};
    ks.hash_kind = KH_BINROW_BIGINT;
    ks.max_p = 128;
    ks.kg_start = 0;
    ks.n_kg = 128;
    ks.sb_per_kg_log2 = 3;
    ks.n_sb = 1024;
    ks.maxp_div = make_udiv32(128);
    const UDiv32 sdiv = make_udiv32(10000);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto go = [&](int i) {
        const int64_t off = (int64_t)(i % NB) * n;
        hipLaunchKernelGGL((k_real<BLOCK, RPT, HIST>), dim3(grid), dim3(BLOCK), 0, 0, k0 + off, t0 + off, v0 + off, out,
                           ks, sdiv, (int64_t)10000);
    };
    for (int i = 0; i < 3; i++) go(i);
    const int reps = 64;
    hipEventRecord(e0, 0);
    for (int i = 0; i < reps; i++) go(i);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / reps;
    printf("%-34s grid %5d  %7.2f us  %6.2f TB/s\n", name, grid, us, n * 24.0 / (us * 1e-6) / 1e12);
}

template <int BLOCK, int RPT, int WORK>
static void run(const char* name, const int64_t* k0, const int64_t* t0, const int64_t* v0, int64_t* out, int64_t n,
                int lds = 0) {
    // NB batches of n rows per column, visited in turn: 2.4 GB, far beyond the 256 MB MALL
    const int grid = (int)(n / (BLOCK * RPT));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto go = [&](int i) {
        const int64_t off = (int64_t)(i % NB) * n;
        hipLaunchKernelGGL((k_probe<BLOCK, RPT, WORK>), dim3(grid), dim3(BLOCK), lds, 0, k0 + off, t0 + off, v0 + off, out);
    };
    for (int i = 0; i < 3; i++) go(i);
    const int reps = 64;
    hipEventRecord(e0, 0);
    for (int i = 0; i < reps; i++) go(i);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / reps;
    printf("%-34s grid %5d  %7.2f us  %6.2f TB/s\n", name, grid, us, n * 24.0 / (us * 1e-6) / 1e12);
}

int main() {
    const int64_t n = 1 << 22;
    int64_t *k, *t, *v, *out;
    hipMalloc(&k, NB * n * 8);
    hipMalloc(&t, NB * n * 8);
    hipMalloc(&v, NB * n * 8);
    hipMalloc(&out, 1 << 20);
    hipMemset(k, 1, NB * n * 8);
    hipMemset(t, 2, NB * n * 8);
    hipMemset(v, 3, NB * n * 8);
    run<512, 8, 0>("512x8 loads only", k, t, v, out, n);
    run<512, 8, 4>("512x8 + 4 mix rounds", k, t, v, out, n);
    run<512, 8, 12>("512x8 + 12 mix rounds", k, t, v, out, n);
    run<256, 8, 0>("256x8 loads only", k, t, v, out, n);
    run<256, 4, 0>("256x4 loads only", k, t, v, out, n);
    run<512, 4, 0>("512x4 loads only", k, t, v, out, n);
    run<1024, 4, 0>("1024x4 loads only", k, t, v, out, n);
    run<256, 16, 0>("256x16 loads only", k, t, v, out, n);
    hipFuncSetAttribute((const void*)k_probe<512, 8, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)k_probe<1024, 4, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)k_probe<512, 4, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    run_real<512, 8, 0>("512x8 real routing", k, t, v, out, n);
    run_real<512, 8, 1>("512x8 real routing + LDS hist", k, t, v, out, n);
    run<512, 8, 0>("512x8 + 78 KB LDS (2/CU)", k, t, v, out, n, 78 * 1024);
    run<512, 8, 0>("512x8 + 52 KB LDS (3/CU)", k, t, v, out, n, 52 * 1024);
    run<512, 8, 0>("512x8 + 39 KB LDS (4/CU)", k, t, v, out, n, 39 * 1024);
    run<512, 4, 0>("512x4 + 39 KB LDS (4/CU)", k, t, v, out, n, 39 * 1024);
    run<1024, 4, 0>("1024x4 + 156 KB LDS (1/CU)", k, t, v, out, n, 156 * 1024);
    hipDeviceSynchronize();
    return 0;
}
