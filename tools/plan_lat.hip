// Latency breakdown of the drop-in plan() below Python: the C ABI sspp_planner_plan per call
// (robocrane, 4096 x 128, as bench.py --mode dropin), and the bare floor of one empty-kernel
// launch + stream synchronisation on the same kind of stream.
//   hipcc --offload-arch=gfx950 -O2 tools/plan_lat.hip -Iinclude -Lsspp_amd/lib -lsspp_hip -o /tmp/plan_lat
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "sspp_hip.h"

__global__ void k_empty(int* p) { if (p && threadIdx.x == 1000) p[0] = 1; }

static double median(std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; }

int main(int argc, char** argv) {
    const char* xml = argc > 1 ? argv[1] : "sspp_amd/scenes/robocrane.xml";
    const int N = 3000;
    using clk = std::chrono::steady_clock;
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    std::vector<double> t;
    for (int grid : {1, 1024}) {
        t.clear();
        for (int i = 0; i < N; ++i) {
            auto a = clk::now();
            hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, st, nullptr);
            hipStreamSynchronize(st);
            t.push_back(std::chrono::duration<double, std::micro>(clk::now() - a).count());
        }
        printf("empty kernel (%d workgroups) launch + stream sync: median %.1f us\n", grid, median(t));
    }
    sspp_model* m = nullptr;
    sspp_scene* s = nullptr;
    sspp_planner* p = nullptr;
    if (sspp_model_load_mjcf(xml, &m) || sspp_scene_create(m, SSPP_MODE_QPOS, 7, 0, &s) || sspp_planner_create(s, 7, &p)) {
        printf("setup failed: %s\n", sspp_last_error());
        return 1;
    }
    const double start[7] = {0.5, 0.15, 0.136, 0.707, 0, 0, 0.707}, end[7] = {0.5, -0.05, 0.136, 0.707, 0, 0, 0.707};
    double lim[7] = {1, 1, 1, 1, 1, 1, 1};
    const int B = 4096, W = 128, n = 10;
    std::vector<double> knots(n + 4), arc(B), ctrl((size_t)B * n * 7);
    std::vector<int64_t> ids(B);
    int64_t nf = 0;
    sspp_best best;
    t.clear();
    for (int i = 0; i < N + 100; ++i) {
        auto a = clk::now();
        if (sspp_planner_plan(p, start, end, 0.08, lim, B, W, n, 0x5EED, 0, knots.data(), &nf, ids.data(), arc.data(),
                              ctrl.data(), &best)) {
            printf("plan failed: %s\n", sspp_last_error());
            return 1;
        }
        if (i >= 100) t.push_back(std::chrono::duration<double, std::micro>(clk::now() - a).count());
    }
    printf("sspp_planner_plan (C ABI, 4096 x 128): median %.1f us, p10 %.1f, feasible %lld, best %lld\n", median(t),
           [&] { auto v = t; std::sort(v.begin(), v.end()); return v[v.size() / 10]; }(), (long long)nf,
           (long long)best.index);
    sspp_planner_free(p);
    sspp_scene_free(s);
    sspp_model_free(m);
    return 0;
}
