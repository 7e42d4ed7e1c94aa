// Same-address vs spread atomic throughput on gfx950 (design input for the
// wavefront queue counters).  hipcc --offload-arch=gfx950 -O3 atomics.hip -o atomics
#include <hip/hip_runtime.h>
#include <cstdio>

// mode 0: all waves -> one u32; 1: one u32 per XCD (blockIdx % 8, 256 B apart);
// 2: one per wave (distinct lines); 3: u64 to one address
__global__ void k_atom(unsigned* c, unsigned long long* c64, int mode, int iters) {
    if ((threadIdx.x & 63u) != 0u) return;
    const unsigned wave = blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u;
    unsigned acc = 0;
    for (int i = 0; i < iters; ++i) {
        if (mode == 0) acc += atomicAdd(c, 1u);
        else if (mode == 1) acc += atomicAdd(c + 64u * (blockIdx.x & 7u), 1u);
        else if (mode == 2) acc += atomicAdd(c + 64u * (wave & 4095u), 1u);
        else acc += (unsigned)atomicAdd(c64, 1ull);
    }
    if (acc == 0xdeadbeefu) c[1] = acc;
}

int main() {
    unsigned* c;
    unsigned long long* c64;
    hipMalloc(&c, 64u * 4096u * 4u);
    hipMalloc(&c64, 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grid = 768, iters = 8;
    for (int mode = 0; mode < 4; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a);
            hipLaunchKernelGGL(k_atom, dim3(grid), dim3(256), 0, 0, c, c64, mode, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double n = (double)grid * 4 * iters;
            if (rep == 2) printf("mode %d: %.0f atomics in %.3f ms = %.1f ns/atomic\n", mode, n, ms, ms * 1e6 / n);
        }
    }
    // empty-kernel launch cost for scale
    hipEventRecord(a);
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_atom, dim3(grid), dim3(256), 0, 0, c, c64, 0, 0);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("empty launch (768x256): %.1f us each\n", ms * 10.0);
    return 0;
}
