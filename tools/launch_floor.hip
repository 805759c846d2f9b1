// Host wall time of one launch + synchronisation of an empty kernel (5120 one-wave workgroups,
// the driver-shaped launch's grid), per stream kind, synchronisation call and scheduling flag.
//   hipcc --offload-arch=gfx950 -O2 tools/launch_floor.hip -o build/launch_floor && build/launch_floor [flag]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

__global__ void k_empty(int* p) { if (p && threadIdx.x == 1023) p[0] = 1; }

static double med(std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; }

int main(int argc, char** argv) {
    const int flag = argc > 1 ? atoi(argv[1]) : -1;  // -1 default, 0 auto, 1 spin, 2 yield, 4 blocking sync
    if (flag >= 0) {
        unsigned f = flag == 0 ? hipDeviceScheduleAuto : flag == 1 ? hipDeviceScheduleSpin
                   : flag == 2 ? hipDeviceScheduleYield : hipDeviceScheduleBlockingSync;
        if (hipSetDeviceFlags(f) != hipSuccess) { printf("hipSetDeviceFlags failed\n"); return 1; }
    }
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int i = 0; i < 20; ++i) { hipLaunchKernelGGL(k_empty, dim3(5120), dim3(64), 0, 0, nullptr); }
    hipDeviceSynchronize();
    const int N = 200;
    for (int mode = 0; mode < 4; ++mode) {  // null+device sync, null+stream sync, own+device, own+stream
        hipStream_t st = mode < 2 ? (hipStream_t)0 : s;
        std::vector<double> t;
        for (int i = 0; i < N; ++i) {
            const auto a = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(k_empty, dim3(5120), dim3(64), 0, st, nullptr);
            if (mode % 2 == 0) hipDeviceSynchronize(); else hipStreamSynchronize(st);
            t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
        }
        printf("flag %d %s stream, %s sync: median %.1f us\n", flag, mode < 2 ? "null" : "own",
               mode % 2 == 0 ? "device" : "stream", med(t));
    }
    return 0;
}
