// Round-trip floor of the resident loops' pod ring: the host posts a doorbell and a
// program of P bytes, G workgroups each see the doorbell and read the program, a device-wide arrival
// counter completes, workgroup 0 writes a result word back; the host times post -> result seen.
//
//   hipcc --offload-arch=gfx950 -O2 -o scripts/ring_latency_probe scripts/ring_latency_probe.hip
//   scripts/ring_latency_probe [G] [P] [iters]
//
// Modes: 0 doorbell + program in coherent host memory, every workgroup polls and reads over PCIe (today's
// ring); 1 as 0 but only workgroup 0 polls host memory, copies the program into device memory and raises a
// device flag the others poll; 2 doorbell + program in fine-grained device memory that the host writes
// directly (large-BAR mapping; the mode is skipped when the host cannot map it); 3 no-op kernel round trip
// via hipLaunchKernel + hipStreamSynchronize, for scale.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

struct Ring {
  unsigned long long ctl;  // posted sequence (0xffffffff: stop)
  unsigned long long pad[15];
  unsigned long long res;  // result sequence
  unsigned long long pad2[15];
  unsigned long long prog[1024];
};

__device__ unsigned long long g_sink;

// every spin is bounded by ~2 s of s_memrealtime (100 MHz)
template <int MODE>
__global__ void __launch_bounds__(256) k_ring(Ring* hr, Ring* dr, unsigned long long* arrive, unsigned long long* flag,
                                              unsigned long long* stage, int P8, int iters) {
  __shared__ unsigned long long s_prog[1024];
  __shared__ int s_go;
  const int t = threadIdx.x;
  const unsigned G = gridDim.x;
  Ring* src = MODE == 2 ? dr : hr;
  for (int q = 1; q <= iters; ++q) {
    if (t == 0) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      int go = 1;
      if (MODE == 1 && blockIdx.x != 0) {
        while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < (unsigned long long)q) {
          if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) { go = 0; break; }
        }
      } else {
        for (;;) {
          const unsigned long long v = __hip_atomic_load(&src->ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if (v == 0xffffffffull) { go = 0; break; }
          if (v >= (unsigned long long)q) break;
          if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) { go = 0; break; }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      s_go = go;
    }
    __syncthreads();
    if (!s_go) return;
    // the program into LDS
    if (MODE == 1 && blockIdx.x != 0) {
      for (int k = t; k < P8; k += 256) s_prog[k] = __hip_atomic_load(stage + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      for (int k = t; k < P8; k += 256) s_prog[k] = __hip_atomic_load(src->prog + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();
    if (MODE == 1 && blockIdx.x == 0) {
      for (int k = t; k < P8; k += 256) __hip_atomic_store(stage + k, s_prog[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      if (t == 0) __hip_atomic_store(flag, (unsigned long long)q, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (t == 0) {
      unsigned long long x = 0;
      for (int k = 0; k < P8; ++k) x += s_prog[k];
      if (x == 12345) g_sink = x;
      __hip_atomic_fetch_add(arrive, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      if (blockIdx.x == 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(arrive, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < (unsigned long long)q * G)
          if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) break;
        __hip_atomic_store(&hr->res, (unsigned long long)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    __syncthreads();
  }
}

__global__ void k_noop() {}

static double run_mode(int mode, int G, int P, int iters, Ring* hr, Ring* hr_dev, Ring* dr, Ring* dr_host) {
  unsigned long long *arrive, *flag, *stage;
  CK(hipMalloc(&arrive, 8));
  CK(hipMalloc(&flag, 8));
  CK(hipMalloc(&stage, 8192));
  CK(hipMemset(arrive, 0, 8));
  CK(hipMemset(flag, 0, 8));
  Ring* w = mode == 2 ? dr_host : hr;  // what the host writes
  __atomic_store_n(&w->ctl, 0ull, __ATOMIC_RELEASE);
  __atomic_store_n(&hr->res, 0ull, __ATOMIC_RELEASE);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int P8 = P / 8;
  if (mode == 0) hipLaunchKernelGGL(k_ring<0>, dim3(G), dim3(256), 0, s, hr_dev, dr, arrive, flag, stage, P8, iters);
  if (mode == 1) hipLaunchKernelGGL(k_ring<1>, dim3(G), dim3(256), 0, s, hr_dev, dr, arrive, flag, stage, P8, iters);
  if (mode == 2) hipLaunchKernelGGL(k_ring<2>, dim3(G), dim3(256), 0, s, hr_dev, dr, arrive, flag, stage, P8, iters);
  std::vector<double> lat;
  std::vector<unsigned long long> prog(P8);
  bool ok = true;
  for (int q = 1; q <= iters && ok; ++q) {
    for (int k = 0; k < P8; ++k) prog[k] = (unsigned long long)q * 1000003ull + k;
    const auto t0 = std::chrono::steady_clock::now();
    std::memcpy(w->prog, prog.data(), (size_t)P8 * 8);
    __atomic_store_n(&w->ctl, (unsigned long long)q, __ATOMIC_RELEASE);
    while (__atomic_load_n(&hr->res, __ATOMIC_ACQUIRE) < (unsigned long long)q) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) { ok = false; break; }
    }
    lat.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  if (!ok) __atomic_store_n(&w->ctl, 0xffffffffull, __ATOMIC_RELEASE);
  CK(hipStreamSynchronize(s));
  CK(hipStreamDestroy(s));
  CK(hipFree(arrive));
  CK(hipFree(flag));
  CK(hipFree(stage));
  if (!ok) return -1;
  std::sort(lat.begin(), lat.end());
  return lat[lat.size() / 2];
}

int main(int argc, char** argv) {
  const int G = argc > 1 ? std::atoi(argv[1]) : 40;
  const int P = argc > 2 ? std::atoi(argv[2]) : 2048;
  const int iters = argc > 3 ? std::atoi(argv[3]) : 2000;
  void* hp = nullptr;
  CK(hipHostMalloc(&hp, sizeof(Ring), hipHostMallocCoherent | hipHostMallocMapped));
  std::memset(hp, 0, sizeof(Ring));
  void* hd = nullptr;
  CK(hipHostGetDevicePointer(&hd, hp, 0));
  Ring* dr = nullptr;
  CK(hipExtMallocWithFlags((void**)&dr, sizeof(Ring), hipDeviceMallocFinegrained));
  CK(hipMemset(dr, 0, sizeof(Ring)));
  CK(hipDeviceSynchronize());
  hipPointerAttribute_t at{};
  const bool host_ok = hipPointerGetAttributes(&at, dr) == hipSuccess && at.hostPointer != nullptr;
  std::printf("{\"G\": %d, \"P\": %d, \"iters\": %d, \"device_ring_host_pointer\": %s", G, P, iters,
              host_ok ? "true" : "false");
  for (int mode = 0; mode < 2; ++mode)
    std::printf(", \"mode%d_median_us\": %.2f", mode, run_mode(mode, G, P, iters, (Ring*)hp, (Ring*)hd, dr, nullptr));
  {  // launch + sync round trip
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<double> lat;
    for (int q = 0; q < 500; ++q) {
      const auto t0 = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(k_noop, dim3(1), dim3(64), 0, s);
      CK(hipStreamSynchronize(s));
      lat.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(lat.begin(), lat.end());
    std::printf(", \"mode3_launch_sync_median_us\": %.2f", lat[lat.size() / 2]);
    CK(hipStreamDestroy(s));
  }
  std::printf("}\n");
  std::fflush(stdout);
  if (host_ok && argc > 4 && std::atoi(argv[4]) == 1) {  // the host writes device memory: last, it may fault
    std::printf("{\"mode2_median_us\": %.2f}\n", run_mode(2, G, P, iters, (Ring*)hp, (Ring*)hd, dr, (Ring*)at.hostPointer));
  }
  return 0;
}
