// Dev probe: the rate of s_memtime (the phase-stamp clock of the PMP_STAMPS builds) against
// s_memrealtime (100 MHz), over a ~20 ms busy loop in one wave.  Build: hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void rate(unsigned long long* out, int iters)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float x = (float)threadIdx.x;
    for (int i = 0; i < iters; i++) x = x * 1.000001f + 0.5f;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = r1 - r0;
        out[2] = (unsigned long long)x;
    }
}

int main()
{
    unsigned long long* d;
    unsigned long long h[3];
    if (hipMalloc(&d, 24) != hipSuccess) return 1;
    for (int iters : {1000000, 4000000}) {
        hipLaunchKernelGGL(rate, dim3(1), dim3(64), 0, 0, d, iters);
        if (hipMemcpy(h, d, 24, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        printf("iters %d: memtime %llu ticks, realtime %llu (100 MHz) -> memtime %.1f MHz\n", iters, h[0], h[1],
               (double)h[0] / ((double)h[1] / 100.0));
    }
    return 0;
}
