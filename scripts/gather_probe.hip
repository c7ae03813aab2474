// gather_probe.hip -- calibration of rocprofv3's FETCH_SIZE on gfx950 for the
// access patterns of this repo's kernels (MI355X_MICROARCH.md: FETCH_SIZE
// reads half the bytes of a 16 B/lane streaming read; other widths are
// uncalibrated).  Every kernel reads a known set of bytes:
//   stream16     : 1 GiB, 16 B per lane, coalesced
//   gather4_hbm  : 2^24 random 4 B reads into 4 GiB (distinct lines w.h.p.,
//                  far past the 256 MiB Infinity Cache)
//   gather8_hbm  : the same with 8 B reads
//   gather4_mall : 2^24 random 4 B reads into 64 MiB (Infinity-Cache resident
//                  after the first touch; launched twice, the second counts)
//   run4_hbm     : 2^24 random 64-lane runs of 4 B (one wave reads 256
//                  contiguous bytes at a random 256 B-aligned place)
// The program prints one JSON line with each launch's time and its known
// read bytes; rocprofv3 --pmc passes over it give FETCH_SIZE per launch.
//   hipcc -O3 --offload-arch=gfx950 -o scripts/bin/gather_probe scripts/gather_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

__global__ void stream16(const float4 *a, uint64_t n4, float *out) {
    float s = 0.f;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.678f) out[0] = s;  // keeps the loads; never true on zeros
}

template <typename T>
__global__ void gather(const T *a, uint64_t n, uint64_t count, uint64_t seed, float *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const T v = a[mix(i + seed) % n];
    if ((float)v == 12345.678f) out[0] = 1.f;
}

__global__ void runs4(const float *a, uint64_t nruns, uint64_t count, float *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint64_t r = mix(i >> 6) % nruns;
    const float v = a[r * 64 + (i & 63)];
    if (v == 12345.678f) out[0] = 1.f;
}

int main() {
    const uint64_t big = 4ull << 30, mall = 64ull << 20, sbytes = 1ull << 30, cnt = 1ull << 24;
    void *p_big = nullptr, *p_mall = nullptr;
    float *out = nullptr;
    CK(hipMalloc(&p_big, big));
    CK(hipMalloc(&p_mall, mall));
    CK(hipMalloc((void **)&out, 64));
    CK(hipMemset(p_big, 0, big));
    CK(hipMemset(p_mall, 0, mall));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned blocks = (unsigned)(cnt / 256);
    std::printf("{\"launches\": [");
    bool first = true;
    auto timed = [&](const char *name, uint64_t bytes, auto launch) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("%s{\"name\": \"%s\", \"known_read_bytes\": %llu, \"ms\": %.4f}", first ? "" : ", ", name,
                    (unsigned long long)bytes, ms);
        first = false;
    };
    timed("stream16", sbytes, [&] { stream16<<<4096, 256>>>((const float4 *)p_big, sbytes / 16, out); });
    timed("gather4_hbm", cnt * 4, [&] { gather<float><<<blocks, 256>>>((const float *)p_big, big / 4, cnt, 1, out); });
    timed("gather8_hbm", cnt * 8,
          [&] { gather<double><<<blocks, 256>>>((const double *)p_big, big / 8, cnt, 2, out); });
    timed("gather4_mall_warm", cnt * 4,
          [&] { gather<float><<<blocks, 256>>>((const float *)p_mall, mall / 4, cnt, 3, out); });
    timed("gather4_mall", cnt * 4, [&] { gather<float><<<blocks, 256>>>((const float *)p_mall, mall / 4, cnt, 3, out); });
    timed("run4_hbm", cnt * 4, [&] { runs4<<<blocks, 256>>>((const float *)p_big, big / 256, cnt, out); });
    std::printf("], \"gather_count\": %llu, \"big_bytes\": %llu, \"mall_bytes\": %llu}\n", (unsigned long long)cnt,
                (unsigned long long)big, (unsigned long long)mall);
    CK(hipFree(p_big));
    CK(hipFree(p_mall));
    CK(hipFree(out));
    return 0;
}
