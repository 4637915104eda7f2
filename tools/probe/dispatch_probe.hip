// dispatch_probe.hip -- analysis only: how many one-wave workgroups the chip keeps resident, and how
// fast it starts them, for waves of a fixed duration.  Each wave spins on s_memrealtime (100 MHz)
// for `ns` nanoseconds and records its start / end; the host reports the peak and mean resident
// count over the launch and the launch time against the ideal (waves x ns / slots).
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/dispatch_probe tools/probe/dispatch_probe.hip
//   tools/probe/dispatch_probe [waves] [ns...]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void __launch_bounds__(64) spin(unsigned long long *rec, unsigned ticks, int lds)
{
    __shared__ unsigned s[64];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (lds) s[threadIdx.x] = threadIdx.x;
    unsigned long long t;
    do t = __builtin_amdgcn_s_memrealtime(); while (t - t0 < ticks);
    if (lds) __builtin_amdgcn_s_barrier();
    if (threadIdx.x == 0) { rec[2 * blockIdx.x] = t0; rec[2 * blockIdx.x + 1] = t + (lds ? s[1] : 0u) * 0u; }
}

int main(int argc, char **argv)
{
    const unsigned waves = argc > 1 ? unsigned(atoi(argv[1])) : 40000u;
    std::vector<unsigned> nss;
    for (int i = 2; i < argc; i++) nss.push_back(unsigned(atoi(argv[i])));
    if (nss.empty()) nss = {2000, 5000, 10000, 20000};
    unsigned long long *d = nullptr;
    if (hipMalloc(&d, sizeof(unsigned long long) * 2 * waves) != hipSuccess) return 1;
    std::vector<unsigned long long> h(2 * size_t(waves));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int lds = 0; lds < 2; lds++)
        for (unsigned ns : nss)
        {
            const unsigned ticks = ns / 10;
            for (int rep = 0; rep < 2; rep++)
            {
                hipEventRecord(a, 0);
                hipLaunchKernelGGL(spin, dim3(waves), dim3(64), 0, 0, d, ticks, lds);
                hipEventRecord(b, 0);
                hipEventSynchronize(b);
            }
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            hipMemcpy(h.data(), d, sizeof(unsigned long long) * 2 * waves, hipMemcpyDeviceToHost);
            unsigned long long lo = ~0ull, hi = 0;
            for (unsigned i = 0; i < waves; i++) { lo = std::min(lo, h[2 * i]); hi = std::max(hi, h[2 * i + 1]); }
            // resident count sampled at 200 points
            std::vector<std::pair<unsigned long long, int>> ev;
            for (unsigned i = 0; i < waves; i++) { ev.push_back({h[2 * i], 1}); ev.push_back({h[2 * i + 1], -1}); }
            std::sort(ev.begin(), ev.end());
            int live = 0, peak = 0;
            double area = 0;
            unsigned long long prev = lo;
            for (auto& e : ev) { area += double(live) * double(e.first - prev); prev = e.first; live += e.second; peak = std::max(peak, live); }
            const double span_ns = double(hi - lo) * 10.0;
            std::printf("{\"lds\": %d, \"wave_ns\": %u, \"waves\": %u, \"kernel_ms\": %.4f, \"span_us\": %.2f, \"ideal_us\": %.2f, "
                        "\"peak_resident\": %d, \"mean_resident\": %.0f, \"start_rate_per_us\": %.1f}\n",
                        lds, ns, waves, ms, span_ns / 1e3, double(waves) * ns / 8192.0 / 1e3, peak,
                        area * 10.0 / span_ns, double(waves) / (span_ns / 1e3));
        }
    return 0;
}
