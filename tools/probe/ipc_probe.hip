// Same-device IPC probe: can two processes on ONE MI355X share a device
// buffer (hipIpcGetMemHandle / hipIpcOpenMemHandle) and hand off flags
// between concurrently running kernels?  This is what the peer-mapped
// record exchange of the distributed LU panel needs on a 2-rank rehearsal
// on one GPU (on 8 GPUs the same handles map peer memory over xGMI).
//
//   ipc_probe 0 <dir> <kind>   exporter: allocates, publishes the handle
//   ipc_probe 1 <dir> <kind>   importer: opens the handle
//   kind: 0 = hipMalloc (coarse grained), 1 = hipDeviceMallocUncached
//
// Both run a one-wave ping-pong kernel (NPING round trips); every spin is
// bounded (a missing peer ends the kernel with a timeout count, never a hang).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <thread>
#include <unistd.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::printf("FAIL %s: %s\n", #x, hipGetErrorString(e_)); std::fflush(stdout); std::exit(2); } } while (0)

constexpr int NPING = 2000;
constexpr long long SPIN = 1ll << 27;     // ~3-4 s of s_sleep(1) polls per wait

__device__ inline long long ld_sys(const long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline void st_sys(long long* p, long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// role 0 answers: waits ping k (slot 0), writes pong k (slot 16 = other line)
// role 1 asks:   writes ping k, waits pong k.  out[0] = timeouts, out[1] = clocks
__global__ void pingpong(long long* box, int role, long long* out) {
    if (threadIdx.x != 0) return;
    long long tmo = 0;
    const long long t0 = clock64();
    for (int k = 1; k <= NPING; ++k) {
        if (role == 1) st_sys(box, k);
        long long* w = role == 0 ? box : box + 16;
        long long s = 0;
        while (ld_sys(w) < k && s < SPIN) { __builtin_amdgcn_s_sleep(1); ++s; }
        if (s >= SPIN) { ++tmo; break; }
        if (role == 0) st_sys(box + 16, k);
    }
    out[0] = tmo;
    out[1] = clock64() - t0;
}

int main(int argc, char** argv) {
    if (argc < 4) { std::printf("usage: ipc_probe role dir kind\n"); return 2; }
    const int role = std::atoi(argv[1]), kind = std::atoi(argv[3]);
    const std::string dir = argv[2], hf = dir + "/handle" + std::to_string(kind);
    CK(hipSetDevice(0));
    long long* box = nullptr;
    hipIpcMemHandle_t h;
    if (role == 0) {
        if (kind == 0) CK(hipMalloc(&box, 1 << 20));
        else CK(hipExtMallocWithFlags((void**)&box, 1 << 20, hipDeviceMallocUncached));
        CK(hipMemset(box, 0, 1 << 20));
        CK(hipDeviceSynchronize());
        CK(hipIpcGetMemHandle(&h, box));
        { std::ofstream f(hf + ".tmp", std::ios::binary); f.write((const char*)&h, sizeof h); }
        std::rename((hf + ".tmp").c_str(), hf.c_str());
        std::printf("role 0 kind %d: exported %p\n", kind, (void*)box);
    } else {
        for (int i = 0; i < 600; ++i) {
            std::ifstream f(hf, std::ios::binary);
            if (f && f.read((char*)&h, sizeof h)) break;
            std::this_thread::sleep_for(std::chrono::milliseconds(50));
            if (i == 599) { std::printf("FAIL no handle file\n"); return 2; }
        }
        CK(hipIpcOpenMemHandle((void**)&box, h, hipIpcMemLazyEnablePeerAccess));
        std::printf("role 1 kind %d: opened %p\n", kind, (void*)box);
    }
    std::fflush(stdout);
    long long* out;
    CK(hipMalloc(&out, 64));
    CK(hipMemset(out, 0, 64));
    const auto w0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(pingpong, dim3(1), dim3(64), 0, 0, box, role, out);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
    long long ho[2];
    CK(hipMemcpy(ho, out, 16, hipMemcpyDeviceToHost));
    std::printf("role %d kind %d: timeouts %lld, %d round trips in %.3f ms wall, %.2f us per round trip (clock64 %lld)\n",
                role, kind, ho[0], NPING, ms, ms * 1e3 / NPING, ho[1]);
    if (role == 1) CK(hipIpcCloseMemHandle(box));
    else {
        std::this_thread::sleep_for(std::chrono::milliseconds(200));
        CK(hipFree(box));
    }
    std::fflush(stdout);
    return ho[0] == 0 ? 0 : 1;
}
