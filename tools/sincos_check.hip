// Dev check: sincos(x) against sin(x) and cos(x) on the device, bit for bit, over atan2's range
// (RRT* steering uses cos(theta) and sin(theta) of one theta).  Build: hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void chk(unsigned long long* bad, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = -3.141592653589793 + 6.283185307179586 * ((double)i + 0.5) / (double)n;
    double s, c;
    sincos(x, &s, &c);
    const double s1 = sin(x), c1 = cos(x);
    if (__double_as_longlong(s) != __double_as_longlong(s1) || __double_as_longlong(c) != __double_as_longlong(c1))
        atomicAdd(bad, 1ull);
}

int main()
{
    unsigned long long* d;
    unsigned long long h = 0;
    if (hipMalloc(&d, 8) != hipSuccess) return 1;
    if (hipMemset(d, 0, 8) != hipSuccess) return 1;
    const int n = 1 << 26;
    hipLaunchKernelGGL(chk, dim3(n / 256), dim3(256), 0, 0, d, n);
    if (hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("sincos vs sin/cos: %llu of %d angles differ\n", h, n);
    return 0;
}
