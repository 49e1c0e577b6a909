/* Can the host store straight into fine-grained device memory (large BAR)?
 * Allocates 4 KiB with hipExtMallocWithFlags(hipDeviceMallocFinegrained),
 * prints its pointer attributes, stores a pattern from the host through the
 * pointer (a segfault here answers "no"), and has a kernel read it back and
 * store a reply the host reads.  Also times host store -> device sees it. */
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>

__global__ void echo(volatile unsigned *p, unsigned rounds)
{
    const unsigned long long t0 = wall_clock64();
    for (unsigned r = 1; r <= rounds; r++) {
        while (__hip_atomic_load((unsigned *)&p[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != r) {
            if (wall_clock64() - t0 > 200000000ull) /* 2 s: give up */
                return;
            __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store((unsigned *)&p[16], r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

int main()
{
    unsigned *p = nullptr;
    if (hipExtMallocWithFlags((void **)&p, 4096, hipDeviceMallocFinegrained) != hipSuccess) {
        std::printf("{\"alloc\": false}\n");
        return 1;
    }
    hipPointerAttribute_t a{};
    (void)hipPointerGetAttributes(&a, p);
    std::printf("type %d device %d hostPointer %p devicePointer %p\n", (int)a.type, a.device, a.hostPointer,
                a.devicePointer);
    std::fflush(stdout);
    hipMemset(p, 0, 4096);
    hipDeviceSynchronize();
    volatile unsigned *vp = p;
    vp[1] = 7; /* segfaults if the host cannot reach it */
    std::printf("host store ok, read back %u\n", vp[1]);
    std::fflush(stdout);
    const unsigned R = 2000;
    hipLaunchKernelGGL(echo, dim3(1), dim3(64), 0, 0, vp, R);
    double tot = 0;
    for (unsigned r = 1; r <= R; r++) {
        const auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n((unsigned *)&p[0], r, __ATOMIC_RELEASE);
        while (__atomic_load_n((unsigned *)&p[16], __ATOMIC_ACQUIRE) != r) {
            __builtin_ia32_pause();
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(3)) {
                std::printf("{\"device_never_answered\": %u}\n", r);
                return 2;
            }
        }
        tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
    hipDeviceSynchronize();
    std::printf("{\"round_trip_us\": %.3f}\n", tot / R);
    /* the same with mapped host memory */
    unsigned *h = nullptr;
    hipHostMalloc((void **)&h, 4096, hipHostMallocMapped | hipHostMallocCoherent);
    std::memset(h, 0, 4096);
    unsigned *hd = nullptr;
    hipHostGetDevicePointer((void **)&hd, h, 0);
    hipLaunchKernelGGL(echo, dim3(1), dim3(64), 0, 0, hd, R);
    tot = 0;
    for (unsigned r = 1; r <= R; r++) {
        const auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(&h[0], r, __ATOMIC_RELEASE);
        while (__atomic_load_n(&h[16], __ATOMIC_ACQUIRE) != r) {
            __builtin_ia32_pause();
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(3))
                return 3;
        }
        tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
    hipDeviceSynchronize();
    std::printf("{\"host_mem_round_trip_us\": %.3f}\n", tot / R);
    return 0;
}
