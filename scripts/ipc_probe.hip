// ipc_probe -- checks the sharded loop's transport on this machine: uncached device memory shared
// over IPC between two processes, granules stored with system scope by one process's kernel and
// polled by the other's.  Usage: ipc_probe server <file> | ipc_probe client <file>.  The server
// allocates, publishes its IPC handle in <file>, then polls for 64 granules; the client opens the
// handle and stores them.  Every spin is bounded; exit status 0 on success.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <thread>

__global__ void k_put(unsigned long long* g, int n, unsigned long long tag) {
  const int i = threadIdx.x;
  if (i < n) __hip_atomic_store(g + i, (tag << 48) | (unsigned long long)(i * 7 + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_poll(const unsigned long long* g, int n, unsigned long long tag, unsigned* ok) {
  const int i = threadIdx.x;
  if (i >= n) return;
  for (unsigned spins = 0; spins < (1u << 24); ++spins) {
    const unsigned long long v = __hip_atomic_load(g + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((v >> 48) == tag && (v & 0xffffffffffffull) == (unsigned long long)(i * 7 + 1)) {
      atomicAdd(ok, 1u);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 2; } } while (0)
int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const int n = 64;
  const unsigned long long tag = 0x1234;
  if (!std::strcmp(argv[1], "server")) {
    void* p = nullptr;
    CK(hipExtMallocWithFlags(&p, 1 << 20, hipDeviceMallocUncached));
    CK(hipMemset(p, 0, 1 << 20));
    hipIpcMemHandle_t h;
    CK(hipIpcGetMemHandle(&h, p));
    unsigned* ok = nullptr;
    CK(hipMalloc(&ok, 4));
    CK(hipMemset(ok, 0, 4));
    hipLaunchKernelGGL(k_poll, dim3(1), dim3(64), 0, 0, (const unsigned long long*)p, n, tag, ok);
    { std::ofstream f(std::string(argv[2]) + ".tmp", std::ios::binary); f.write((const char*)&h, sizeof h); }
    std::rename((std::string(argv[2]) + ".tmp").c_str(), argv[2]);
    CK(hipDeviceSynchronize());
    unsigned got = 0;
    CK(hipMemcpy(&got, ok, 4, hipMemcpyDeviceToHost));
    std::printf("server: %u of %d granules seen\n", got, n);
    return got == (unsigned)n ? 0 : 1;
  }
  hipIpcMemHandle_t h;
  for (int k = 0; k < 600; ++k) {
    std::ifstream f(argv[2], std::ios::binary);
    if (f && f.read((char*)&h, sizeof h)) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
    if (k == 599) { std::fprintf(stderr, "client: no handle\n"); return 2; }
  }
  void* q = nullptr;
  CK(hipIpcOpenMemHandle(&q, h, hipIpcMemLazyEnablePeerAccess));
  hipLaunchKernelGGL(k_put, dim3(1), dim3(64), 0, 0, (unsigned long long*)q, n, tag);
  CK(hipDeviceSynchronize());
  CK(hipIpcCloseMemHandle(q));
  std::printf("client: stored %d granules\n", n);
  return 0;
}
