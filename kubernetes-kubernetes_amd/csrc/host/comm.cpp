// comm.cpp -- RCCL and in-process transports of the node-sharded exchange (comm.hpp).
#include "comm.hpp"

#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <string>
#include <map>
#include <mutex>
#include <vector>

#include "../common/desc.h"
#include "host.hpp"

namespace ksg {

hipError_t launch_max_reduce(unsigned long long* dst, const RankPtrs& src, int nsrc, int count, hipStream_t s);

// ---------------------------------------------------------------------------------------------
// RCCL: one process per GPU (bench.py under torch.distributed.run); ncclMax over uint64.
// ---------------------------------------------------------------------------------------------
class RcclComm : public Comm {
 public:
  ncclComm_t comm = nullptr;
  int all_reduce_max(unsigned long long* buf, size_t count, hipStream_t s) override {
    const ncclResult_t r = ncclAllReduce(buf, buf, count, ncclUint64, ncclMax, comm, s);
    if (r != ncclSuccess) {
      err = std::string("ncclAllReduce: ") + ncclGetErrorString(r);
      return KSG_EDEVICE;
    }
    return KSG_OK;
  }
  int group_begin() override { return ncclGroupStart() == ncclSuccess ? KSG_OK : KSG_EDEVICE; }
  int group_end() override { return ncclGroupEnd() == ncclSuccess ? KSG_OK : KSG_EDEVICE; }
  std::vector<void*> opened;  // peers' IPC mappings (closed on destruction)
  ~RcclComm() override;
  // IPC handles all-gathered over RCCL, then opened (hipIpcOpenMemHandle maps the peer GPU's memory)
  int share_buffers(void* mine, std::vector<void*>* all) override {
    hipIpcMemHandle_t h;
    if (hipIpcGetMemHandle(&h, mine) != hipSuccess) {
      err = "hipIpcGetMemHandle failed";
      return KSG_EDEVICE;
    }
    const size_t hb = sizeof(hipIpcMemHandle_t);
    char* d = nullptr;
    hipStream_t s = nullptr;
    std::vector<char> hostv((size_t)world * hb);
    if (hipMalloc(&d, (size_t)world * hb) != hipSuccess || hipStreamCreate(&s) != hipSuccess) {
      err = "share_buffers: allocation failed";
      return KSG_EDEVICE;
    }
    int rc = KSG_OK;
    if (hipMemcpy(d + (size_t)rank * hb, &h, hb, hipMemcpyHostToDevice) != hipSuccess ||
        ncclAllGather(d + (size_t)rank * hb, d, hb, ncclChar, comm, s) != ncclSuccess ||
        hipStreamSynchronize(s) != hipSuccess ||
        hipMemcpy(hostv.data(), d, (size_t)world * hb, hipMemcpyDeviceToHost) != hipSuccess) {
      err = "share_buffers: handle all-gather failed";
      rc = KSG_EDEVICE;
    }
    (void)hipFree(d);
    (void)hipStreamDestroy(s);
    if (rc) return rc;
    all->assign(world, nullptr);
    for (int r = 0; r < world; ++r) {
      if (r == rank) {
        (*all)[r] = mine;
        continue;
      }
      hipIpcMemHandle_t ph;
      std::memcpy(&ph, hostv.data() + (size_t)r * hb, hb);
      void* p = nullptr;
      if (hipIpcOpenMemHandle(&p, ph, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
        err = "hipIpcOpenMemHandle failed for rank " + std::to_string(r);
        return KSG_EDEVICE;
      }
      opened.push_back(p);
      (*all)[r] = p;
    }
    return KSG_OK;
  }
};
RcclComm::~RcclComm() {
  for (void* p : opened) (void)hipIpcCloseMemHandle(p);
  if (comm) (void)ncclCommDestroy(comm);
}

static bool hex_to_id(const std::string& hex, ncclUniqueId* id) {
  if (hex.size() != 2 * sizeof(id->internal)) return false;
  for (size_t i = 0; i < sizeof(id->internal); ++i) {
    unsigned v = 0;
    if (std::sscanf(hex.c_str() + 2 * i, "%2x", &v) != 1) return false;
    id->internal[i] = (char)v;
  }
  return true;
}

int comm_unique_id(std::string* hex, std::string* err) {
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    *err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
    return KSG_EDEVICE;
  }
  hex->clear();
  char b[3];
  for (size_t i = 0; i < sizeof(id.internal); ++i) {
    std::snprintf(b, sizeof b, "%02x", (unsigned)(unsigned char)id.internal[i]);
    *hex += b;
  }
  return KSG_OK;
}

// ---------------------------------------------------------------------------------------------
// Local: `world` contexts in one process on one device, each driven by its own host thread.
// Every exchange is a host rendezvous at ENQUEUE time (no device synchronisation): each rank
// records an event after its producer kernel, the ranks swap (vector, event) pairs, and each
// rank's stream waits for the other ranks' events before its max-reduce kernel.
// ---------------------------------------------------------------------------------------------
struct LocalGroup {
  std::mutex mu;
  std::condition_variable cv;
  int world = 0, arrived = 0, members = 0;
  uint64_t gen = 0;
  hipEvent_t launched = nullptr;  // group_launch: the leader's event after the group's dispatch
  int launch_rc = 0;              // ... and the leader's status
  std::vector<unsigned long long*> bufs;
  std::vector<hipEvent_t> evs;
  std::vector<size_t> counts;
  // snapshot of each completed generation (two alternate: a rank can be at most one ahead)
  std::vector<unsigned long long*> snap_bufs[2];
  std::vector<hipEvent_t> snap_evs[2];
  bool count_mismatch[2] = {false, false};
};

static std::mutex g_groups_mu;
static std::map<std::string, std::shared_ptr<LocalGroup>> g_groups;

class LocalComm : public Comm {
 public:
  std::string name;
  std::shared_ptr<LocalGroup> g;
  static constexpr int kRing = 4;  // events per rank (rank skew is at most one exchange)
  hipEvent_t ring[kRing] = {};
  int next_ev = 0;

  ~LocalComm() override {
    for (hipEvent_t e : ring)
      if (e) (void)hipEventDestroy(e);
    if (launched) (void)hipEventDestroy(launched);
    std::lock_guard<std::mutex> lk(g_groups_mu);
    if (g && --g->members == 0) g_groups.erase(name);
  }

  // all ranks arrive; returns false on timeout (a rank stopped issuing the same sequence)
  bool rendezvous(unsigned long long* buf, hipEvent_t ev, size_t count, int* slot) {
    std::unique_lock<std::mutex> lk(g->mu);
    const uint64_t my = g->gen;
    g->bufs[rank] = buf;
    g->evs[rank] = ev;
    g->counts[rank] = count;
    if (++g->arrived == g->world) {
      const int sl = (int)(my & 1u);
      g->snap_bufs[sl] = g->bufs;
      g->snap_evs[sl] = g->evs;
      bool mism = false;
      for (size_t c : g->counts) mism |= c != g->counts[0];
      g->count_mismatch[sl] = mism;
      g->arrived = 0;
      ++g->gen;
      g->cv.notify_all();
    } else if (!g->cv.wait_for(lk, std::chrono::seconds(120), [&] { return g->gen != my; })) {
      return false;
    }
    *slot = (int)(my & 1u);
    return !g->count_mismatch[*slot];
  }

  int all_reduce_max(unsigned long long* buf, size_t count, hipStream_t s) override {
    hipEvent_t ev = ring[next_ev];
    next_ev = (next_ev + 1) % kRing;
    if (hipEventRecord(ev, s) != hipSuccess) {
      err = "local exchange: hipEventRecord failed";
      return KSG_EDEVICE;
    }
    int sl = 0;
    if (!rendezvous(buf, ev, count, &sl)) {
      err = "local exchange: ranks did not issue the same exchange sequence (timeout or size mismatch)";
      return KSG_EDEVICE;
    }
    RankPtrs src{};
    for (int r = 0; r < world; ++r) {
      src.p[r] = g->snap_bufs[sl][r];
      if (r != rank && hipStreamWaitEvent(s, g->snap_evs[sl][r], 0) != hipSuccess) {
        err = "local exchange: hipStreamWaitEvent failed";
        return KSG_EDEVICE;
      }
    }
    if (launch_max_reduce(buf, src, world, (int)count, s) != hipSuccess) {
      err = "local exchange: reduce launch failed";
      return KSG_EDEVICE;
    }
    return KSG_OK;
  }

  int share_buffers(void* mine, std::vector<void*>* all) override {  // one process: the pointers themselves
    int sl = 0;
    if (!rendezvous((unsigned long long*)mine, nullptr, 0, &sl)) {
      err = "local exchange: buffer rendezvous timed out";
      return KSG_EDEVICE;
    }
    all->assign(world, nullptr);
    for (int r = 0; r < world; ++r) (*all)[r] = g->snap_bufs[sl][r];
    return KSG_OK;
  }

  bool in_process() const override { return true; }

  hipEvent_t launched = nullptr;  // the leader's (rank 0's) group_launch event
  int group_launch(void* req, hipStream_t s, const GroupLaunchFn& leader) override {
    hipEvent_t ev = ring[next_ev];
    next_ev = (next_ev + 1) % kRing;
    if (hipEventRecord(ev, s) != hipSuccess) {  // everything this rank enqueued before its loop
      err = "group launch: hipEventRecord failed";
      return KSG_EDEVICE;
    }
    int sl = 0;
    if (!rendezvous(reinterpret_cast<unsigned long long*>(req), ev, 0, &sl)) {
      err = "group launch: ranks did not issue the same launch sequence (timeout)";
      return KSG_EDEVICE;
    }
    if (rank == 0) {  // every rank is blocked in the second rendezvous until this is enqueued
      std::vector<void*> reqs(world);
      int rc = KSG_OK;
      for (int r = 0; r < world; ++r) {
        reqs[r] = g->snap_bufs[sl][r];
        if (r && hipStreamWaitEvent(s, g->snap_evs[sl][r], 0) != hipSuccess) rc = KSG_EDEVICE;
      }
      if (!launched && hipEventCreateWithFlags(&launched, hipEventDisableTiming) != hipSuccess) rc = KSG_EDEVICE;
      if (rc == KSG_OK) rc = leader(s, reqs);
      if (rc == KSG_OK && hipEventRecord(launched, s) != hipSuccess) rc = KSG_EDEVICE;
      std::lock_guard<std::mutex> lk(g->mu);
      g->launched = launched;
      g->launch_rc = rc;
    }
    if (!rendezvous(nullptr, nullptr, 0, &sl)) {
      err = "group launch: launch rendezvous timed out";
      return KSG_EDEVICE;
    }
    int rc;
    hipEvent_t done;
    {
      std::lock_guard<std::mutex> lk(g->mu);
      rc = g->launch_rc;
      done = g->launched;
    }
    if (rc != KSG_OK) {
      err = "group launch: the leader could not enqueue the group's dispatch";
      return KSG_EDEVICE;
    }
    // (the leader records `launched` again only after every rank has passed the next first rendezvous)
    if (rank != 0 && hipStreamWaitEvent(s, done, 0) != hipSuccess) {
      err = "group launch: hipStreamWaitEvent failed";
      return KSG_EDEVICE;
    }
    return KSG_OK;
  }

  int agree(int64_t mine, std::vector<int64_t>* all) override {
    int64_t v = mine;
    int sl = 0;
    if (!rendezvous(reinterpret_cast<unsigned long long*>(&v), nullptr, 0, &sl)) {
      err = "local exchange: outcome rendezvous timed out";
      return KSG_EDEVICE;
    }
    all->assign(world, 0);
    for (int r = 0; r < world; ++r) (*all)[r] = *reinterpret_cast<const int64_t*>(g->snap_bufs[sl][r]);
    if (!rendezvous(nullptr, nullptr, 0, &sl)) {  // every rank has read the others' values (on their stacks)
      err = "local exchange: outcome rendezvous timed out";
      return KSG_EDEVICE;
    }
    return KSG_OK;
  }

  int launch_gate() override {
    int sl = 0;
    if (!rendezvous(nullptr, nullptr, 0, &sl)) {
      err = "local exchange: launch rendezvous timed out";
      return KSG_EDEVICE;
    }
    return KSG_OK;
  }

  int batch_end() override {  // every rank's stream has drained: buffers may be reused/regrown
    int sl = 0;
    if (!rendezvous(nullptr, nullptr, 0, &sl)) {
      err = "local exchange: batch-end rendezvous timed out";
      return KSG_EDEVICE;
    }
    return KSG_OK;
  }
};

std::unique_ptr<Comm> make_comm(const Config& cfg, std::string* err) {
  if (!cfg.sharded()) return nullptr;
  if (!cfg.nccl_id.empty()) {
    ncclUniqueId id;
    if (!hex_to_id(cfg.nccl_id, &id)) {
      *err = "distributed.ncclId must be the 256 hex characters of ksg_comm_unique_id";
      return nullptr;
    }
    auto c = std::make_unique<RcclComm>();
    c->world = cfg.world;
    c->rank = cfg.rank;
    const ncclResult_t r = ncclCommInitRank(&c->comm, cfg.world, id, cfg.rank);
    if (r != ncclSuccess) {
      c->comm = nullptr;
      *err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
      return nullptr;
    }
    return c;
  }
  auto c = std::make_unique<LocalComm>();
  c->world = cfg.world;
  c->rank = cfg.rank;
  c->name = cfg.local_group;
  for (hipEvent_t& e : c->ring)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      *err = "local exchange: hipEventCreate failed";
      return nullptr;
    }
  {
    std::lock_guard<std::mutex> lk(g_groups_mu);
    auto& g = g_groups[cfg.local_group];
    if (!g) {
      g = std::make_shared<LocalGroup>();
      g->world = cfg.world;
      g->bufs.assign(cfg.world, nullptr);
      g->evs.assign(cfg.world, nullptr);
      g->counts.assign(cfg.world, 0);
    }
    if (g->world != cfg.world || g->members >= cfg.world) {
      *err = "local exchange group '" + cfg.local_group + "': worldSize mismatch or rank already joined";
      return nullptr;
    }
    ++g->members;
    c->g = g;
  }
  return c;
}

}  // namespace ksg
