// Probe: does a stream wait on a value that kernels on other streams advance
// (hipStreamWaitValue64 on hipMallocSignalMemory), also while another stream's
// kernel is still running? Used to decide how k_chain_ci's progress gates the
// path stage (render.hip). Exits 0 when every check passes; each wait is
// bounded by the host watchdog below (the process exits with 3 if a wait hangs).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>

__global__ void k_bump(unsigned long long* sig, int spin_us) {
    // every workgroup: spin a little, then add 1 to the signal (system scope)
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < (long long)spin_us * 100) __builtin_amdgcn_s_sleep(8);
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(sig, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_record(const unsigned long long* sig, unsigned long long* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *out = __hip_atomic_load(sig, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main() {
    int can = 0;
    (void)hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0);
    printf("hipDeviceAttributeCanUseStreamWaitValue = %d\n", can);
    unsigned long long* sig = nullptr;
    hipError_t e = hipExtMallocWithFlags((void**)&sig, sizeof(unsigned long long), hipMallocSignalMemory);
    printf("hipExtMallocWithFlags(signal) = %s\n", hipGetErrorString(e));
    if (e != hipSuccess) return 1;
    unsigned long long* out = nullptr;
    (void)hipMalloc((void**)&out, 8);
    hipStream_t a, b;
    (void)hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
    std::thread watchdog([] {
        std::this_thread::sleep_for(std::chrono::seconds(40));
        printf("watchdog: a wait hung\n");
        fflush(stdout);
        std::_Exit(3);
    });
    watchdog.detach();
    for (int round = 0; round < 3; round++) {
        const unsigned long long base = round * 1000ull;
        // stream b waits for 1000 bumps beyond base, then records the value
        e = hipStreamWaitValue64(b, sig, base + 1000, hipStreamWaitValueGte);
        if (e != hipSuccess) { printf("hipStreamWaitValue64: %s\n", hipGetErrorString(e)); return 1; }
        hipLaunchKernelGGL(k_record, dim3(1), dim3(64), 0, b, sig, out);
        // stream a: 1000 workgroups bump it over ~ a few ms
        hipLaunchKernelGGL(k_bump, dim3(1000), dim3(64), 0, a, sig, 50);
        const auto t0 = std::chrono::steady_clock::now();
        (void)hipStreamSynchronize(b);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        (void)hipStreamSynchronize(a);
        unsigned long long v = 0;
        (void)hipMemcpy(&v, out, 8, hipMemcpyDeviceToHost);
        printf("round %d: b saw %llu (want >= %llu) after %.2f ms\n", round, v, base + 1000, ms);
        if (v < base + 1000) return 2;
    }
    printf("ok\n");
    return 0;
}
