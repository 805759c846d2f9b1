// Host wall time of one launch + completion wait of an empty kernel (1024 four-wave workgroups,
// the single-step plan() grid), per stream kind, wait and scheduling flag.  Wait modes:
//   device / stream: hipDeviceSynchronize / hipStreamSynchronize after the launch;
//   flag: the last workgroup to finish (one device-scope counter per launch) stores a sequence
//   number into mapped pinned host memory after a system-scope fence, and the host spins on it.
//   hipcc --offload-arch=gfx950 -O2 tools/launch_floor.hip -o tools/launch_floor.bin && tools/launch_floor.bin [flag]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_empty(int* p) { if (p && threadIdx.x == 1023) p[0] = 1; }

// every workgroup arrives once; the last one re-arms the counter and publishes `seq`
__global__ void k_empty_flag(unsigned* count, volatile unsigned* host_flag, unsigned seq) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gridDim.x - 1) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __threadfence_system();
            __hip_atomic_store((unsigned*)host_flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

static double med(std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; }

int main(int argc, char** argv) {
    const int flag = argc > 1 ? atoi(argv[1]) : -1;  // -1 default, 0 auto, 1 spin, 2 yield, 4 blocking sync
    if (flag >= 0) {
        unsigned f = flag == 0 ? hipDeviceScheduleAuto : flag == 1 ? hipDeviceScheduleSpin
                   : flag == 2 ? hipDeviceScheduleYield : hipDeviceScheduleBlockingSync;
        if (hipSetDeviceFlags(f) != hipSuccess) { printf("hipSetDeviceFlags failed\n"); return 1; }
    }
    const int nblk = 1024, nthr = 256;
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k_empty, dim3(nblk), dim3(nthr), 0, 0, nullptr);
    hipDeviceSynchronize();
    const int N = 200;
    for (int mode = 0; mode < 4; ++mode) {  // null+device sync, null+stream sync, own+device, own+stream
        hipStream_t st = mode < 2 ? (hipStream_t)0 : s;
        std::vector<double> t;
        for (int i = 0; i < N; ++i) {
            const auto a = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(k_empty, dim3(nblk), dim3(nthr), 0, st, nullptr);
            if (mode % 2 == 0) hipDeviceSynchronize(); else hipStreamSynchronize(st);
            t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
        }
        printf("flag %d %s stream, %s sync: median %.1f us\n", flag, mode < 2 ? "null" : "own",
               mode % 2 == 0 ? "device" : "stream", med(t));
    }
    // completion flag in mapped pinned memory, host spin
    unsigned* d_count = nullptr;
    unsigned* h_flag = nullptr;
    unsigned* d_flag = nullptr;
    hipMalloc((void**)&d_count, sizeof(unsigned));
    hipMemset(d_count, 0, sizeof(unsigned));
    hipHostMalloc((void**)&h_flag, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent);
    hipHostGetDevicePointer((void**)&d_flag, h_flag, 0);
    *h_flag = 0;
    hipDeviceSynchronize();
    std::vector<double> t;
    for (unsigned i = 1; i <= (unsigned)N; ++i) {
        const auto a = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(k_empty_flag, dim3(nblk), dim3(nthr), 0, s, d_count, d_flag, i);
        while (std::atomic_ref<unsigned>(*h_flag).load(std::memory_order_acquire) != i) {
        }
        t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
    }
    hipStreamSynchronize(s);
    printf("flag %d own stream, host spin on a mapped completion flag: median %.1f us\n", flag, med(t));
    hipFree(d_count);
    hipHostFree(h_flag);
    return 0;
}
