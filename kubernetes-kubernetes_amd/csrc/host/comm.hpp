// comm.hpp -- the per-pod exchange of the node-sharded scheduler.
//
// Each rank evaluates a contiguous block range of the snapshot order; per pod the ranks
// all-reduce (MAX) small fixed-layout uint64 vectors (desc.h XaWord/XpWord/XbWord): feasible
// counts, NormalizeScore maxima/minima, PodTopologySpread domain presence, and the packed
// (TotalScore, heap pre-order key) + node of every rank's best node.  The exchange is
// stream-ordered: it is enqueued between the kernels of a pod, so a whole batch of pods runs
// without a host round trip.
//
// Two transports behind one interface:
//   RcclComm  -- one process per GPU, RCCL ncclAllReduce(ncclUint64, ncclMax) over xGMI.
//   LocalComm -- ranks in one process sharing one device (threads, one context each); the
//                all-reduce is an event-ordered max-reduce kernel reading every rank's vector.
//                This is how the sharded path is exercised on a single-GPU box.
#pragma once
#include <hip/hip_runtime.h>

#include <functional>
#include <memory>
#include <string>
#include <vector>

namespace ksg {

struct Config;

class Comm {
 public:
  virtual ~Comm() = default;
  int world = 1, rank = 0;
  // in-stream all-reduce(MAX) of `count` uint64 words at device pointer `buf`, in place
  virtual int all_reduce_max(unsigned long long* buf, size_t count, hipStream_t s) = 0;
  // brackets several all-reduces that may be fused (ncclGroupStart/End)
  virtual int group_begin() { return 0; }
  virtual int group_end() { return 0; }
  // end of a batch: every rank's stream has drained (already synchronised by the caller)
  virtual int batch_end() { return 0; }
  // before a batch's first persistent-loop launch: in-process ranks share one device, and a rank
  // still in a synchronising HIP call (allocation, first use) must not hold its loop back while
  // a peer's loop is already spinning on it
  virtual int launch_gate() { return 0; }
  // collective: every rank passes its device buffer; all[r] becomes rank r's buffer as mapped in
  // this process (in-process: the pointer itself; RCCL ranks: an IPC mapping of the peer's memory)
  virtual int share_buffers(void* mine, std::vector<void*>* all) = 0;
  // In-process groups (one device): every rank's persistent loop goes into ONE dispatch (DESIGN.md §6:
  // loops dispatched separately on separate hardware queues are not co-scheduled).  Each rank passes its
  // launch request (`req`, valid until the call returns); the leader (rank 0) makes its stream wait for every
  // rank's stream, calls leader(its stream, every rank's req) to enqueue the group's dispatch, and every other
  // rank's stream then waits for that.  RCCL ranks (a device each) launch their own loops and never call this.
  using GroupLaunchFn = std::function<int(hipStream_t, const std::vector<void*>&)>;
  virtual int group_launch(void* req, hipStream_t s, const GroupLaunchFn& leader) {
    err = "group_launch: only in-process groups launch their loops together";
    return -1;
  }
  virtual bool in_process() const { return false; }
  // host-side: all[r] = rank r's `mine` (in-process groups; the RCCL transport has no host channel and
  // returns only its own value)
  virtual int agree(int64_t mine, std::vector<int64_t>* all) {
    all->assign(1, mine);
    return 0;
  }
  std::string err;
};

// nullptr + *err on failure; cfg.world == 1 never creates one
std::unique_ptr<Comm> make_comm(const Config& cfg, std::string* err);
// ncclGetUniqueId as 256 hex characters (rank 0 creates it and hands it to every rank)
int comm_unique_id(std::string* hex, std::string* err);

}  // namespace ksg
