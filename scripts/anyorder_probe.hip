// Does hipExtAnyOrderLaunch let a dispatch start while the dispatch before it on the SAME stream still runs
// (the AQL barrier bit cleared)?  Kernel A spins until kernel B, launched after it on the same stream, sets a
// flag; every spin is bounded (2 s of s_memrealtime), so a serialised pair ends with A timing out.
//   hipcc --offload-arch=gfx950 -O2 -o scripts/anyorder_probe scripts/anyorder_probe.hip && ./scripts/anyorder_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_wait(unsigned* flag, unsigned* out) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned seen = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < 200000000ull) {  // 2 s
    seen = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (seen) break;
    __builtin_amdgcn_s_sleep(2);
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = seen ? (unsigned)((__builtin_amdgcn_s_memrealtime() - t0) / 100) + 1 : 0u;
}
__global__ void k_set(unsigned* flag) {
  if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int main() {
  unsigned *flag, *out;
  hipStream_t s;
  if (hipMalloc(&flag, 4) || hipMalloc(&out, 4) || hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) return 2;
  for (int mode = 0; mode < 2; ++mode) {
    unsigned h = 0;
    (void)hipMemset(flag, 0, 4);
    (void)hipMemset(out, 0, 4);
    (void)hipDeviceSynchronize();
    hipExtLaunchKernelGGL(k_wait, dim3(4), dim3(64), 0, s, nullptr, nullptr, 0, flag, out);
    hipExtLaunchKernelGGL(k_set, dim3(1), dim3(64), 0, s, nullptr, nullptr, mode ? hipExtAnyOrderLaunch : 0, flag);
    if (hipStreamSynchronize(s) != hipSuccess) return 3;
    (void)hipMemcpy(&h, out, 4, hipMemcpyDeviceToHost);
    std::printf("%s: %s\n", mode ? "second dispatch with hipExtAnyOrderLaunch" : "second dispatch in order",
                h ? "ran while the first still spun" : "waited for the first to end (it timed out after 2 s)");
  }
  return 0;
}
