// cache_events.cpp -- sanitizer harness (test infrastructure, built only by tests/asan/Makefile with
// -fsanitize=address,undefined): seeded cache-event sequences through the product's host cache shadow
// (csrc/host/cluster.cpp: Cache.AddNode / UpdateNode / RemoveNode / AddPod / RemovePod and the assume / forget of
// a compiled pod; csrc/host/podtable.cpp: the pod table's precompile, slot reservation, drop and upload; the
// mirror's re-layout and in-place update staging) with the HIP runtime stubbed over host memory
// (hip_host_stub.cpp), and the same events through the parity oracle.  After every event the return codes must
// agree, and after every "mirror" event the snapshot order (UpdateSnapshot, cache.go:190-296) must equal the
// oracle's.
// Usage: cache_events <events file: "<op>\t<arg>[\t<arg2>]" per line> [config json]
//   node|upd <node json>   rmnode <name>   pod <bound pod json>   rmpod <uid>
//   assume <unbound pod json> <node> <uid>: the compiled pod's slot (pod_table_precompile + pod_table_put), then
//          the AssumePod of Engine::run_batch (add_pod with the uid and node overrides)
//   forget <uid>   drop <pod json>: a slot reserved and released unplaced (a failed compile)
//   mirror: ensure_mirror + the pod table's upload, then the snapshot order against the oracle's
// Exit status 0 unless an event diverged (1) or a sanitizer reported (its own abort).
#include <cstdio>
#include <fstream>
#include <string>
#include <vector>

#include "host.hpp"
#include "../../oracle/ksg_oracle.h"

static std::vector<std::string> split(const std::string& s) {
  std::vector<std::string> out;
  size_t a = 0;
  for (size_t b; (b = s.find('\t', a)) != std::string::npos; a = b + 1) out.push_back(s.substr(a, b - a));
  out.push_back(s.substr(a));
  return out;
}

// the JSON of a pod with spec.nodeName and metadata.uid set (the oracle's form of an assumed pod)
static std::string bind_json(const std::string& j, const std::string& node, const std::string& uid) {
  std::string o = j;
  const size_t spec = o.find("\"spec\":{");
  if (spec == std::string::npos) return o;
  o.insert(spec + 8, "\"nodeName\":\"" + node + "\",");
  const size_t u = o.find("\"uid\":\"");
  if (u != std::string::npos) {
    const size_t e = o.find('"', u + 7);
    o.replace(u + 7, e - (u + 7), uid);
  }
  return o;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: cache_events <events> [config json]\n");
    return 2;
  }
  const std::string cfgj = argc > 2 ? argv[2] : "{}";
  ksg::Config cfg;
  std::string err;
  if (!ksg::decode_config(cfgj.data(), cfgj.size(), &cfg, &err)) {
    std::fprintf(stderr, "config: %s\n", err.c_str());
    return 2;
  }
  ksg::Cluster c(cfg);
  ksgo_ctx* o = ksgo_create(cfgj.data(), cfgj.size());
  if (!o) return 2;
  std::ifstream in(argv[1]);
  std::string line;
  long events = 0, mirrors = 0, bad = 0;
  while (std::getline(in, line)) {
    const std::vector<std::string> f = split(line);
    const std::string& op = f[0];
    int rp = KSG_OK, ro = KSG_OK;
    if (op == "node" || op == "upd") {
      ksg::NodeSpec n;
      if (!ksg::decode_node(f[1].data(), f[1].size(), &n, &err)) continue;
      rp = op == "node" ? c.add_node(std::move(n)) : c.update_node(std::move(n));
      ro = op == "node" ? ksgo_add_node(o, f[1].data(), f[1].size()) : ksgo_update_node(o, f[1].data(), f[1].size());
    } else if (op == "rmnode") {
      rp = c.remove_node(f[1]);
      ro = ksgo_remove_node(o, f[1].c_str());
    } else if (op == "pod") {
      ksg::PodSpec p;
      if (!ksg::decode_pod(f[1].data(), f[1].size(), &p, &err)) continue;
      rp = c.add_pod(p);
      ro = ksgo_add_pod(o, f[1].data(), f[1].size());
    } else if (op == "rmpod" || op == "forget") {
      rp = c.remove_pod(f[1]);
      ro = ksgo_remove_pod(o, f[1].c_str());
    } else if (op == "assume") {
      ksg::PodSpec p;
      if (!ksg::decode_pod(f[1].data(), f[1].size(), &p, &err)) continue;
      c.pod_table_precompile(p);
      const int32_t slot = c.pod_table_put(p, -1);
      rp = c.add_pod(p, f[3], false, slot, &f[2]);
      if (rp != KSG_OK) c.pod_table_drop(slot);
      const std::string b = bind_json(f[1], f[2], f[3]);
      ro = ksgo_add_pod(o, b.data(), b.size());
    } else if (op == "drop") {
      ksg::PodSpec p;
      if (!ksg::decode_pod(f[1].data(), f[1].size(), &p, &err)) continue;
      c.pod_table_precompile(p);
      c.pod_table_drop(c.pod_table_put(p, -1));
    } else if (op == "mirror") {
      ++mirrors;
      rp = c.ensure_mirror(true);
      if (rp == KSG_OK) rp = c.upload_pod_table(false);
      const std::vector<std::string>& ord = c.order();
      const int no = ksgo_num_nodes(o);
      bool same = no == (int)ord.size();
      char buf[512];
      for (int i = 0; same && i < no; ++i) {
        ksgo_node_name(o, i, buf, sizeof buf);
        same = ord[(size_t)i] == buf;
      }
      if (!same) {
        std::fprintf(stderr, "event %ld: snapshot order differs from the oracle's (%zu vs %d nodes)\n", events, ord.size(), no);
        ++bad;
      }
    } else {
      continue;
    }
    if ((rp == KSG_OK) != (ro == KSG_OK)) {
      std::fprintf(stderr, "event %ld (%s): product rc %d, oracle rc %d (%s | %s)\n", events, op.c_str(), rp, ro,
                   c.err.c_str(), ksgo_last_error(o));
      ++bad;
    }
    c.err.clear();
    ++events;
  }
  ksgo_destroy(o);
  std::printf("%ld events, %ld mirror checks, %ld divergences\n", events, mirrors, bad);
  return bad ? 1 : 0;
}
