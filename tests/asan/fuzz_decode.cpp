// fuzz_decode.cpp -- sanitizer harness (test infrastructure, built only by tests/asan/Makefile with
// -fsanitize=address,undefined): seeded JSON mutations through the product's host decode
// (kubernetes-kubernetes_amd/csrc/host/objects.cpp over json.hpp: what ksg_pod_compile / ksg_add_node /
// ksg_upsert_namespace / ksg_upsert_object / ksg_create decode from caller-supplied bytes) and through the
// parity oracle's identical C API (oracle/: decode, cache events and scheduling cycles on the CPU).
// Usage: fuzz_decode <corpus: one JSON document per line, "<kind>\t<json>"> <seed> <mutations per document>
// Exit status 0 unless a sanitizer reports (ASan / UBSan abort the process with their own report).
#include <cstdio>
#include <cstdint>
#include <fstream>
#include <random>
#include <string>
#include <vector>

#include "host.hpp"
#include "../../oracle/ksg_oracle.h"

namespace {

std::string mutate(const std::string& s, std::mt19937_64& rng) {
  std::string o = s;
  const int ops = 1 + (int)(rng() % 4);
  static const char* kTokens[] = {"{", "}", "[", "]", ",", ":", "\"", "null", "true", "-1", "1e309", "\"\\u00",
                                  "\"a\"", "0.5", "\"99999999999999999999\"", "{\"\":[]}", "\\", "\"cpu\"", "\"1Gi\""};
  for (int k = 0; k < ops && !o.empty(); ++k) {
    const size_t at = rng() % (o.size() + 1);
    switch (rng() % 6) {
      case 0: o.erase(at, 1 + rng() % 8); break;                                   // drop bytes
      case 1: o.insert(at, kTokens[rng() % (sizeof(kTokens) / sizeof(*kTokens))]); break;  // a token
      case 2: if (at < o.size()) o[at] = (char)(rng() % 256); break;                // a byte
      case 3: o = o.substr(0, at); break;                                          // truncate
      case 4: {                                                                    // duplicate a span
        const size_t len = 1 + rng() % 32;
        if (at < o.size()) o.insert(at, o.substr(at, len));
        break;
      }
      default: {                                                                   // swap two spans
        const size_t b = rng() % (o.size() + 1), len = 1 + rng() % 16;
        if (at + len <= o.size() && b + len <= o.size()) for (size_t i = 0; i < len; ++i) std::swap(o[at + i], o[b + i]);
      }
    }
  }
  return o;
}

void product_decode(const std::string& kind, const std::string& j) {
  std::string err;
  if (kind == "pod") {
    ksg::PodSpec p;
    if (ksg::decode_pod(j.data(), j.size(), &p, &err)) {
      (void)ksg::calc_resources(p);
      (void)ksg::calc_fit_request(p);
    }
  } else if (kind == "node") {
    ksg::NodeSpec n;
    (void)ksg::decode_node(j.data(), j.size(), &n, &err);
  } else if (kind == "ns") {
    ksg::NamespaceSpec n;
    (void)ksg::decode_namespace(j.data(), j.size(), &n, &err);
  } else if (kind == "obj") {
    ksg::SelectorObj o;
    (void)ksg::decode_selector_obj(j.data(), j.size(), &o, &err);
  } else if (kind == "config") {
    ksg::Config c;
    (void)ksg::decode_config(j.data(), j.size(), &c, &err);
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  std::ifstream in(argv[1]);
  std::vector<std::pair<std::string, std::string>> docs;
  for (std::string line; std::getline(in, line);) {
    const size_t tab = line.find('\t');
    if (tab != std::string::npos) docs.push_back({line.substr(0, tab), line.substr(tab + 1)});
  }
  std::mt19937_64 rng(std::stoull(argv[2]));
  const int per = std::stoi(argv[3]);
  // the oracle: one context fed the unmutated cluster, then mutated events and cycles
  ksgo_ctx* o = ksgo_create("{}", 2);
  size_t decoded = 0, oracle_ok = 0;
  for (auto& d : docs) {
    if (d.first == "node") ksgo_add_node(o, d.second.data(), d.second.size());
    if (d.first == "ns") ksgo_upsert_namespace(o, d.second.data(), d.second.size());
  }
  for (auto& d : docs) {
    for (int k = 0; k <= per; ++k) {
      const std::string j = k == 0 ? d.second : mutate(d.second, rng);
      product_decode(d.first, j);
      ++decoded;
      int32_t h = -1;
      int rc = -1;
      if (d.first == "pod") {
        rc = ksgo_pod_compile(o, j.data(), j.size(), &h);
        if (rc == KSG_OK) {
          ksg_result r;
          rc = ksgo_schedule_one(o, h, 0, &r, nullptr);
          ksgo_pod_release(o, h);
        }
      } else if (d.first == "node") {
        rc = ksgo_update_node(o, j.data(), j.size());
      } else if (d.first == "ns") {
        rc = ksgo_upsert_namespace(o, j.data(), j.size());
      } else if (d.first == "obj") {
        rc = ksgo_upsert_object(o, j.data(), j.size());
      } else if (d.first == "config") {
        ksgo_ctx* c = ksgo_create(j.data(), j.size());
        rc = c ? KSG_OK : -1;
        if (c) ksgo_destroy(c);
      }
      oracle_ok += rc == KSG_OK;
    }
  }
  ksgo_destroy(o);
  std::printf("fuzz_decode: %zu documents decoded by both, %zu accepted by the oracle\n", decoded, oracle_ok);
  return 0;
}
