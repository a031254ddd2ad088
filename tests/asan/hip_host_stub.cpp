// hip_host_stub.cpp -- test infrastructure for the host-only sanitizer build of the cache shadow
// (tests/asan/Makefile, cache_events): the HIP runtime calls cluster.cpp and podtable.cpp make, over host memory
// (allocations are calloc, copies memcpy, streams and synchronisation no-ops), and the four mirror-maintenance
// kernels they launch (k_node_update, k_node_dyn, k_gather_rows, k_gather_csr) as no-ops.  Nothing here models
// the device: the harness checks the host side -- the cache events' shadow, the snapshot order, the pod table and
// the staging the uploads pack -- against the oracle, under AddressSanitizer and UndefinedBehaviorSanitizer.
#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <cstring>

#include "../../kubernetes-kubernetes_amd/csrc/common/desc.h"

extern "C" {
hipError_t hipSetDevice(int) { return hipSuccess; }
const char* hipGetErrorString(hipError_t) { return "hip host stub"; }
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned int) {
  *s = reinterpret_cast<hipStream_t>(std::malloc(8));  // a distinct handle, freed by hipStreamDestroy
  return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
  std::free(s);
  return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipMalloc(void** p, size_t n) {
  *p = std::calloc(1, n ? n : 1);
  return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void* p) {
  std::free(p);
  return hipSuccess;
}
hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) {
  if (n) std::memmove(d, s, n);
  return hipSuccess;
}
hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t) {
  if (n) std::memmove(d, s, n);
  return hipSuccess;
}
}

namespace ksg {
hipError_t launch_node_update(const MirrorView&, const NodeUpdate*, const uint32_t*, const LabelEntry*, const ScalarEntry*,
                              int, hipStream_t) {
  return hipSuccess;
}
hipError_t launch_node_dyn(const MirrorView&, const NodeDyn*, const uint32_t*, const ScalarEntry*, int, hipStream_t) {
  return hipSuccess;
}
hipError_t launch_gather_rows(uint8_t*, const uint8_t*, const int32_t*, int, int, int, int, hipStream_t) { return hipSuccess; }
hipError_t launch_gather_csr(uint32_t*, const uint32_t*, const int32_t*, const uint32_t*, const uint32_t*, int, hipStream_t) {
  return hipSuccess;
}
}  // namespace ksg
