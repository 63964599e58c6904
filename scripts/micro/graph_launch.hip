// Launch cost of a small batch's kernel chain: K dependent tiny kernels per iteration, timed as
//   direct   : K hipLaunchKernelGGL + hipStreamSynchronize
//   capture  : the same K launches under stream capture, hipGraphExecUpdate of the cached executable
//              graph (instantiated once), hipGraphLaunch + hipStreamSynchronize
//   replay   : hipGraphLaunch of an unchanged executable graph + hipStreamSynchronize
// hipcc --offload-arch=gfx950 -O3 scripts/micro/graph_launch.hip -o scripts/micro/graph_launch
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void tiny(uint32_t *buf, uint32_t n, uint32_t add)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) buf[i] += add;
}

int main(int argc, char **argv)
{
    const int K = argc > 1 ? atoi(argv[1]) : 32, IT = argc > 2 ? atoi(argv[2]) : 300;
    const uint32_t n = 1u << 14;
    uint32_t *buf = nullptr;
    CK(hipMalloc(&buf, n * 4 * 4));
    CK(hipMemset(buf, 0, n * 16));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    auto chain = [&](uint32_t it) {
        for (int k = 0; k < K; ++k)
            hipLaunchKernelGGL(tiny, dim3(16 + (k % 4) * 16), dim3(256), 0, st, buf + (k % 4) * n, n, it + k);
    };
    using clk = std::chrono::steady_clock;
    // warm up
    for (int i = 0; i < 20; ++i) chain(i);
    CK(hipStreamSynchronize(st));
    auto t0 = clk::now();
    for (int i = 0; i < IT; ++i) { chain(i); CK(hipStreamSynchronize(st)); }
    const double direct = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / IT;

    hipGraph_t g = nullptr;
    hipGraphExec_t ex = nullptr;
    double cap_us = 0, upd_us = 0, launch_us = 0;
    t0 = clk::now();
    for (int i = 0; i < IT + 5; ++i) {
        if (i == 5) t0 = clk::now();
        auto a = clk::now();
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
        chain(i);
        hipGraph_t gi = nullptr;
        CK(hipStreamEndCapture(st, &gi));
        auto b = clk::now();
        if (!ex) {
            CK(hipGraphInstantiate(&ex, gi, nullptr, nullptr, 0));
        } else {
            hipGraphExecUpdateResult r;
            hipGraphNode_t en = nullptr;
            if (hipGraphExecUpdate(ex, gi, &en, &r) != hipSuccess) {
                fprintf(stderr, "update failed (%d): re-instantiate\n", (int)r);
                CK(hipGraphExecDestroy(ex));
                CK(hipGraphInstantiate(&ex, gi, nullptr, nullptr, 0));
            }
        }
        auto c = clk::now();
        CK(hipGraphLaunch(ex, st));
        CK(hipStreamSynchronize(st));
        auto d = clk::now();
        if (g) CK(hipGraphDestroy(g));
        g = gi;
        if (i >= 5) {
            cap_us += std::chrono::duration<double, std::micro>(b - a).count();
            upd_us += std::chrono::duration<double, std::micro>(c - b).count();
            launch_us += std::chrono::duration<double, std::micro>(d - c).count();
        }
    }
    const double capture = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / IT;
    t0 = clk::now();
    for (int i = 0; i < IT; ++i) { CK(hipGraphLaunch(ex, st)); CK(hipStreamSynchronize(st)); }
    const double replay = std::chrono::duration<double, std::micro>(clk::now() - t0).count() / IT;
    printf("{\"kernels\": %d, \"iterations\": %d, \"direct_us\": %.1f, \"capture_update_launch_us\": %.1f, "
           "\"capture_us\": %.1f, \"update_us\": %.1f, \"launch_sync_us\": %.1f, \"replay_us\": %.1f}\n",
           K, IT, direct, capture, cap_us / IT, upd_us / IT, launch_us / IT, replay);
    return 0;
}
