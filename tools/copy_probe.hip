// tools/copy_probe.hip -- which float4 copy reaches the achievable HBM rate
// (the bench's hbm_copy_GBps reference); prints GB/s (read + write) per
// variant, best of 10.  hipcc --offload-arch=gfx950 -O3 -o copy_probe copy_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_k(const u32x4 *__restrict__ a, u32x4 *__restrict__ b, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        u32x4 x[U];
#pragma unroll
        for (int k = 0; k < U; ++k) x[k] = NT ? __builtin_nontemporal_load(a + i + k * stride) : a[i + k * stride];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (NT) __builtin_nontemporal_store(x[k], b + i + k * stride);
            else b[i + k * stride] = x[k];
        }
    }
    for (; i < n; i += stride) b[i] = a[i];
}

// one block owns a contiguous span, lanes interleaved
template <int U>
__global__ void __launch_bounds__(256) copy_span(const u32x4 *__restrict__ a, u32x4 *__restrict__ b, uint64_t n,
                                                 uint64_t per) {
    const uint64_t s0 = (uint64_t)blockIdx.x * per, s1 = s0 + per < n ? s0 + per : n;
    for (uint64_t i = s0 + threadIdx.x; i < s1; i += U * 256) {
        u32x4 x[U];
#pragma unroll
        for (int k = 0; k < U; ++k) if (i + k * 256 < s1) x[k] = a[i + k * 256];
#pragma unroll
        for (int k = 0; k < U; ++k) if (i + k * 256 < s1) b[i + k * 256] = x[k];
    }
}

int main() {
    const uint64_t bytes = 1ull << 31;
    const uint64_t n = bytes / 16;
    u32x4 *a, *b;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMemset(a, 1, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char *name, auto launch) {
        float best = 1e9;
        for (int r = 0; r < 11; ++r) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (r && ms < best) best = ms;
        }
        printf("%-28s %8.1f GB/s\n", name, 2.0 * bytes / (best * 1e-3) / 1e9);
    };
    timeit("hipMemcpyDtoD", [&] { hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0); });
    const unsigned grids[] = {1024, 2048, 4096, 8192, 16384, 65536};
    for (unsigned g : grids) {
        char nm[64];
        snprintf(nm, sizeof nm, "u1 g%u", g);
        timeit(nm, [&] { copy_k<1, false><<<g, 256>>>(a, b, n); });
        snprintf(nm, sizeof nm, "u4 g%u", g);
        timeit(nm, [&] { copy_k<4, false><<<g, 256>>>(a, b, n); });
        snprintf(nm, sizeof nm, "u4nt g%u", g);
        timeit(nm, [&] { copy_k<4, true><<<g, 256>>>(a, b, n); });
        snprintf(nm, sizeof nm, "u8 g%u", g);
        timeit(nm, [&] { copy_k<8, false><<<g, 256>>>(a, b, n); });
    }
    for (unsigned g : {1024u, 2048u, 4096u, 8192u}) {
        char nm[64];
        snprintf(nm, sizeof nm, "span4 g%u", g);
        const uint64_t per = (n + g - 1) / g;
        timeit(nm, [&] { copy_span<4><<<g, 256>>>(a, b, n, per); });
    }
    unsigned g = (unsigned)(n / 256);
    timeit("u1 one-per-thread", [&] { copy_k<1, false><<<g, 256>>>(a, b, n); });
    return 0;
}
