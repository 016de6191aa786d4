// Latency probe for the single-workgroup sweep kernel's building blocks on gfx950: one 256-thread
// workgroup timing (wall clock, 100 MHz) a barrier, a dependent LDS load, a dependent global load
// (L2-resident), s_memrealtime itself and a dependent fp64 divide.
//   hipcc --offload-arch=gfx950 -O3 -o lat_probe scripts/lat_probe.hip && ./lat_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(256) void probe(int* chain, double* out, int iters) {
    __shared__ int lds[1024];
    for (int i = threadIdx.x; i < 1024; i += 256) lds[i] = (i * 7 + 1) & 1023;
    __syncthreads();
    unsigned long long t0, t1;
    // 1. barrier
    t0 = wall_clock64();
    for (int i = 0; i < iters; ++i) __syncthreads();
    t1 = wall_clock64();
    if (threadIdx.x == 0) out[0] = (double)(t1 - t0) * 10.0 / iters;  // ns
    // 2. dependent LDS loads
    int x = threadIdx.x & 1023;
    t0 = wall_clock64();
    for (int i = 0; i < iters; ++i) x = lds[x];
    t1 = wall_clock64();
    if (threadIdx.x == 0) out[1] = (double)(t1 - t0) * 10.0 / iters;
    // 3. dependent global loads (a 4 KiB chain: L2 / L1 resident after the first lap)
    int y = threadIdx.x & 1023;
    for (int i = 0; i < 1024; ++i) y = chain[y];
    t0 = wall_clock64();
    for (int i = 0; i < iters; ++i) y = chain[y];
    t1 = wall_clock64();
    if (threadIdx.x == 0) out[2] = (double)(t1 - t0) * 10.0 / iters;
    // 4. the clock read
    unsigned long long acc = 0;
    t0 = wall_clock64();
    for (int i = 0; i < iters; ++i) acc += wall_clock64();
    t1 = wall_clock64();
    if (threadIdx.x == 0) out[3] = (double)(t1 - t0) * 10.0 / iters;
    // 5. dependent fp64 divides
    double d = 1.0 + threadIdx.x * 1e-3;
    t0 = wall_clock64();
    for (int i = 0; i < iters; ++i) d = 1.0000001 / d;
    t1 = wall_clock64();
    if (threadIdx.x == 0) out[4] = (double)(t1 - t0) * 10.0 / iters;
    // 6. shader clock ticks per wall tick
    unsigned long long c0 = clock64();
    t0 = wall_clock64();
    for (int i = 0; i < iters; ++i) d = d * 1.0000001;
    unsigned long long c1 = clock64();
    t1 = wall_clock64();
    if (threadIdx.x == 0) {
        out[5] = (double)(c1 - c0) / ((double)(t1 - t0) * 10.0);  // GHz
        out[6] = d + (double)(x + y) + (double)acc * 0.0;
    }
}

int main() {
    int* chain;
    double* out;
    hipMalloc(&chain, 1024 * sizeof(int));
    hipMallocManaged(&out, 8 * sizeof(double));
    int h[1024];
    for (int i = 0; i < 1024; ++i) h[i] = (i * 193 + 7) & 1023;
    hipMemcpy(chain, h, sizeof(h), hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(256), 0, 0, chain, out, 2000);
        hipDeviceSynchronize();
        printf("barrier %.1f ns | LDS dep load %.1f ns | global dep load %.1f ns | wall_clock64 %.1f ns | "
               "fp64 div %.1f ns | shader clock %.2f GHz\n",
               out[0], out[1], out[2], out[3], out[4], out[5]);
    }
    return 0;
}
