// Does the runtime pass kernel arguments larger than 4 KiB intact?  The output pointer comes FIRST
// so a truncated argument block can only garble the values read, never the store's address.
// hipcc --offload-arch=gfx950 -O2 -o tools/probe/kernarg_probe tools/probe/kernarg_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
struct Big { float v[2048]; };   // 8 KiB
__global__ void k(float *o, Big b) { o[threadIdx.x] = b.v[(threadIdx.x * 37u) % 2048u]; }
int main()
{
    static Big b;
    for (int i = 0; i < 2048; i++) b.v[i] = float(i);
    float *d = nullptr;
    if (hipMalloc(&d, 4 * 64) != hipSuccess) return 2;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, b);
    hipError_t e = hipGetLastError();
    hipError_t e2 = hipDeviceSynchronize();
    float h[64] = {};
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 3;
    int bad = 0;
    for (int t = 0; t < 64; t++) bad += h[t] != float((t * 37) % 2048);
    std::printf("{\"launch\": \"%s\", \"sync\": \"%s\", \"bad\": %d, \"h63\": %.1f}\n", hipGetErrorString(e),
                hipGetErrorString(e2), bad, h[63]);
    return bad ? 1 : 0;
}
