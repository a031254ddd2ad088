// objects.cpp -- v1 object decoding and the O(pod) helper semantics the compiler needs.
#include <algorithm>
#include <climits>

#include "host.hpp"

namespace ksg {

// ---- resource.Quantity -> milli-units (apimachinery/pkg/api/resource/quantity.go) ------------
// The value is held exactly as digits * 2^b2 * 10^e10 and scaled to milli with a
// round-up (MilliValue / ScaledValue semantics).
bool parse_quantity(const std::string& s, int64_t* milli) {
  const char* p = s.c_str();
  const char* e = p + s.size();
  int sign = 1;
  if (p < e && (*p == '+' || *p == '-')) sign = (*p++ == '-') ? -1 : 1;
  unsigned __int128 digits = 0;
  int frac_digits = 0, nd = 0;
  bool seen_dot = false;
  for (; p < e; ++p) {
    if (*p >= '0' && *p <= '9') {
      if (digits > ((unsigned __int128)1 << 96)) return false;
      digits = digits * 10u + (unsigned)(*p - '0');
      nd++;
      if (seen_dot) frac_digits++;
    } else if (*p == '.' && !seen_dot) {
      seen_dot = true;
    } else {
      break;
    }
  }
  if (nd == 0) return false;
  const std::string suffix(p, e);
  int b2 = 0, e10 = 0;
  if (suffix.empty()) {
  } else if (suffix.size() == 2 && suffix[1] == 'i') {
    static const char* bin = "KMGTPE";
    const char* q = std::strchr(bin, suffix[0]);
    if (!q) return false;
    b2 = 10 * (int)(q - bin + 1);
  } else if (suffix.size() == 1) {
    switch (suffix[0]) {
      case 'n': e10 = -9; break;
      case 'u': e10 = -6; break;
      case 'm': e10 = -3; break;
      case 'k': e10 = 3; break;
      case 'M': e10 = 6; break;
      case 'G': e10 = 9; break;
      case 'T': e10 = 12; break;
      case 'P': e10 = 15; break;
      case 'E': e10 = 18; break;
      default: return false;
    }
  } else if (suffix[0] == 'e' || suffix[0] == 'E') {
    int64_t x;
    if (!parse_go_int(suffix.substr(1), &x) || x < -40 || x > 40) return false;
    e10 = (int)x;
  } else {
    return false;
  }
  const unsigned __int128 cap = (unsigned __int128)1 << 120;
  unsigned __int128 v = digits << b2;
  int scale = e10 - frac_digits + 3;
  for (; scale > 0; --scale) {
    v *= 10u;
    if (v > cap) { *milli = sign > 0 ? LLONG_MAX : LLONG_MIN; return true; }
  }
  if (scale < 0) {
    unsigned __int128 d = 1;
    for (; scale < 0 && d < cap; ++scale) d *= 10u;
    v = sign > 0 ? (v + d - 1) / d : v / d;
  }
  if (v > (unsigned __int128)LLONG_MAX) v = LLONG_MAX;
  *milli = sign > 0 ? (int64_t)v : -(int64_t)v;
  return true;
}

int64_t milli_ceil(int64_t m) { return m >= 0 ? m / 1000 + (m % 1000 ? 1 : 0) : m / 1000; }

bool parse_go_int(const std::string& s, int64_t* v) {
  if (s.empty()) return false;
  size_t i = (s[0] == '+' || s[0] == '-') ? 1 : 0;
  if (i == s.size()) return false;
  const bool neg = s[0] == '-';
  unsigned __int128 acc = 0;
  for (; i < s.size(); ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    acc = acc * 10 + (unsigned)(s[i] - '0');
    if (acc > (unsigned __int128)LLONG_MAX + 1) return false;
  }
  if (!neg && acc > (unsigned __int128)LLONG_MAX) return false;
  *v = neg ? (int64_t)(-(__int128)acc) : (int64_t)acc;
  return true;
}

// ---- validation (apimachinery/pkg/util/validation/validation.go) -----------------------------
static bool alnum(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); }
static bool qualified_name_part(const std::string& s) {
  if (s.empty() || s.size() > 63 || !alnum(s.front()) || !alnum(s.back())) return false;
  return std::all_of(s.begin(), s.end(), [](char c) { return alnum(c) || c == '-' || c == '_' || c == '.'; });
}
static bool dns_subdomain(const std::string& s) {
  if (s.empty() || s.size() > 253) return false;
  size_t i = 0;
  while (i <= s.size()) {
    size_t j = s.find('.', i);
    if (j == std::string::npos) j = s.size();
    if (j == i) return false;
    auto low = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
    if (!low(s[i]) || !low(s[j - 1])) return false;
    for (size_t k = i; k < j; ++k)
      if (!low(s[k]) && s[k] != '-') return false;
    i = j + 1;
  }
  return true;
}
bool valid_label_key(const std::string& k) {
  size_t sl = k.find('/');
  if (sl == std::string::npos) return qualified_name_part(k);
  if (k.find('/', sl + 1) != std::string::npos) return false;
  return dns_subdomain(k.substr(0, sl)) && qualified_name_part(k.substr(sl + 1));
}
bool valid_label_value(const std::string& v) { return v.empty() || qualified_name_part(v); }

bool scalar_resource(const std::string& n) {  // v1helper Is{Extended,HugePage,PrefixedNative,AttachableVolume}
  const bool prefixed_native = n.find("kubernetes.io/") != std::string::npos;
  const bool native = n.find('/') == std::string::npos || prefixed_native;
  const bool extended = !native && n.rfind("requests.", 0) != 0 && valid_label_key("requests." + n);
  return extended || n.rfind("hugepages-", 0) == 0 || prefixed_native || n.rfind("attachable-volumes-", 0) == 0;
}

// ---- JSON decoding ------------------------------------------------------------------------
static StrMap kv_map(const JDoc& d, const JVal* o) {
  StrMap m;
  d.each(o, [&](const JVal& v) {
    if (v.type == JVal::STR) m.emplace_back(v.key, v.s);
  });
  std::sort(m.begin(), m.end());
  return m;
}
static std::vector<std::string> str_list(const JDoc& d, const JVal* a) {
  std::vector<std::string> out;
  d.each(a, [&](const JVal& v) {
    if (v.type == JVal::STR) out.push_back(v.s);
  });
  return out;
}
static bool res_list(const JDoc& d, const JVal* o, ResVec* out, std::string* err) {
  bool ok = true;
  d.each(o, [&](const JVal& v) {
    int64_t m;
    if (!ok) return;
    if (!parse_quantity(v.s, &m)) {
      *err = "invalid quantity " + v.key + "=" + v.s;
      ok = false;
      return;
    }
    out->push_back({v.key, m});
  });
  return ok;
}
static std::vector<Expr> exprs(const JDoc& d, const JVal* a) {
  std::vector<Expr> out;
  d.each(a, [&](const JVal& e) { out.push_back({d.str(e, "key"), d.str(e, "operator"), str_list(d, d.get(e, "values"))}); });
  return out;
}
static NSTerm ns_term(const JDoc& d, const JVal& t) {
  return NSTerm{exprs(d, d.get(t, "matchExpressions")), exprs(d, d.get(t, "matchFields"))};
}
static LabelSel label_sel(const JDoc& d, const JVal* v) {
  LabelSel s;
  if (!v) return s;
  s.present = true;
  s.match = kv_map(d, d.get(*v, "matchLabels"));
  s.exprs = exprs(d, d.get(*v, "matchExpressions"));
  return s;
}
static PATerm pa_term(const JDoc& d, const JVal& t, int32_t weight) {
  PATerm p;
  p.sel = label_sel(d, d.get(t, "labelSelector"));
  p.namespaces = str_list(d, d.get(t, "namespaces"));
  p.ns_sel = label_sel(d, d.get(t, "namespaceSelector"));
  p.topo = d.str(t, "topologyKey");
  p.weight = weight;
  return p;
}
static bool container(const JDoc& d, const JVal& c, Container* out, std::string* err) {
  out->name = d.str(c, "name");
  out->image = d.str(c, "image");
  if (const JVal* r = d.get(c, "resources"))
    if (!res_list(d, d.get(*r, "requests"), &out->req, err)) return false;
  d.each(d.get(c, "ports"), [&](const JVal& p) {
    out->ports.push_back({d.str(p, "hostIP"), d.str(p, "protocol"), (int32_t)d.num(p, "hostPort")});
  });
  out->sidecar = d.str(c, "restartPolicy") == "Always";
  return true;
}

// metav1.Time's RFC 3339 text ("2006-01-02T15:04:05Z", optional fraction up to 9 digits, Z or
// +hh:mm / -hh:mm) to Unix nanoseconds; days from the civil date by the proleptic Gregorian rule
bool parse_rfc3339(const std::string& s, int64_t* unix_ns) {
  auto dig = [&](size_t at, int n, int64_t* v) {
    if (at + n > s.size()) return false;
    int64_t x = 0;
    for (int k = 0; k < n; ++k) {
      const char ch = s[at + k];
      if (ch < '0' || ch > '9') return false;
      x = x * 10 + (ch - '0');
    }
    *v = x;
    return true;
  };
  int64_t Y, M, D, h, mi, sec;
  if (!dig(0, 4, &Y) || s.size() < 20 || s[4] != '-' || !dig(5, 2, &M) || s[7] != '-' || !dig(8, 2, &D) ||
      (s[10] != 'T' && s[10] != 't') || !dig(11, 2, &h) || s[13] != ':' || !dig(14, 2, &mi) || s[16] != ':' ||
      !dig(17, 2, &sec))
    return false;
  size_t q = 19;
  int64_t frac = 0;
  if (q < s.size() && s[q] == '.') {
    int nd = 0;
    for (++q; q < s.size() && s[q] >= '0' && s[q] <= '9'; ++q, ++nd)
      if (nd < 9) frac = frac * 10 + (s[q] - '0');
    if (nd == 0) return false;
    for (int k = nd; k < 9; ++k) frac *= 10;
  }
  int64_t off = 0;
  if (q < s.size() && (s[q] == 'Z' || s[q] == 'z')) {
    ++q;
  } else if (q < s.size() && (s[q] == '+' || s[q] == '-')) {
    int64_t oh, om;
    if (!dig(q + 1, 2, &oh) || q + 3 >= s.size() || s[q + 3] != ':' || !dig(q + 4, 2, &om)) return false;
    off = (s[q] == '-' ? -1 : 1) * (oh * 3600 + om * 60);
    q += 6;
  } else {
    return false;
  }
  if (q != s.size() || M < 1 || M > 12 || D < 1 || D > 31 || h > 23 || mi > 59 || sec > 60) return false;
  const int64_t y = Y - (M <= 2);  // days_from_civil
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const int64_t yoe = y - era * 400;
  const int64_t doy = (153 * (M + (M > 2 ? -3 : 9)) + 2) / 5 + D - 1;
  const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  const int64_t days = era * 146097 + doe - 719468;
  *unix_ns = ((days * 86400 + h * 3600 + mi * 60 + sec) - off) * 1000000000LL + frac;
  return true;
}

// every request / overhead names cpu, memory or ephemeral-storage only (PodSpec::scalar_free)
bool pod_scalar_free(const PodSpec& p) {
  auto ok = [](const ResVec& v) {
    for (auto& r : v)
      if (r.name != "cpu" && r.name != "memory" && r.name != "ephemeral-storage") return false;
    return true;
  };
  for (auto& k : p.containers)
    if (!ok(k.req) || !ok(k.st_req) || !ok(k.st_alloc)) return false;
  for (auto& k : p.init_containers)
    if (!ok(k.req) || !ok(k.st_req) || !ok(k.st_alloc)) return false;
  return ok(p.pod_requests) && ok(p.overhead) && ok(p.pod_st_req) && ok(p.pod_st_alloc);
}
static void pod_sign_fragments(const JDoc& d, const JVal& root, PodSpec* out);  // below

bool decode_pod(const char* p, size_t n, PodSpec* out, std::string* err) {
  try {
    JDoc d(p, n);
    const JVal& r = d.root();
    const JVal* md = d.get(r, "metadata");
    if (!md) { *err = "pod without metadata"; return false; }
    out->name = d.str(*md, "name");
    out->ns = d.str(*md, "namespace", "default");
    if (out->ns.empty()) out->ns = "default";  // apiserver defaulting of metadata.namespace
    out->uid = d.str(*md, "uid");
    if (out->uid.empty()) out->uid = out->ns + "/" + out->name;
    out->labels = kv_map(d, d.get(*md, "labels"));
    out->terminating = d.present(*md, "deletionTimestamp");
    // metav1.GetControllerOfNoCopy (apimachinery/pkg/apis/meta/v1/controller_ref.go): the first
    // ownerReference with controller == true
    d.each(d.get(*md, "ownerReferences"), [&](const JVal& o) {
      if (out->has_controller || !d.boolean(o, "controller")) return;
      out->has_controller = true;
      out->owner_api = d.str(o, "apiVersion");
      out->owner_kind = d.str(o, "kind");
      out->owner_name = d.str(o, "name");
    });
    // container statuses by name (AggregateContainerRequests' map: containerStatuses, then
    // initContainerStatuses over them), kept while their resources are non-nil
    struct CStat { std::string name; bool res; ResVec req, alloc; };
    std::vector<CStat> cstats;
    if (const JVal* st = d.get(r, "status")) {
      bool ok = true;
      for (const char* key : {"containerStatuses", "initContainerStatuses"})
        d.each(d.get(*st, key), [&](const JVal& cs) {
          CStat x{d.str(cs, "name"), false, {}, {}};
          if (const JVal* rs = d.get(cs, "resources")) {
            x.res = true;
            ok = ok && res_list(d, d.get(*rs, "requests"), &x.req, err);
          }
          ok = ok && res_list(d, d.get(cs, "allocatedResources"), &x.alloc, err);
          cstats.push_back(std::move(x));
        });
      if (const JVal* rs = d.get(*st, "resources")) {
        out->has_pod_status_res = true;
        ok = ok && res_list(d, d.get(*rs, "requests"), &out->pod_st_req, err);
        ok = ok && res_list(d, d.get(*st, "allocatedResources"), &out->pod_st_alloc, err);
      }
      // IsPodResizeInfeasible (helpers.go:311-320): the first PodResizePending condition decides
      bool seen_resize = false;
      d.each(d.get(*st, "conditions"), [&](const JVal& c) {
        if (seen_resize || d.str(c, "type") != "PodResizePending") return;
        seen_resize = true;
        out->resize_infeasible = d.str(c, "reason") == "Infeasible";
      });
      if (!ok) return false;
      const std::string t = d.str(*st, "startTime");
      if (!t.empty()) {
        if (!parse_rfc3339(t, &out->start_ns)) { *err = "bad status.startTime " + t; return false; }
        out->has_start = true;
      }
      out->nominated_node = d.str(*st, "nominatedNodeName");
      // PodTerminatingByPreemption (preemption/util.go:23-35): the first DisruptionTarget condition decides
      bool seen = false;
      d.each(d.get(*st, "conditions"), [&](const JVal& c) {
        if (seen || d.str(c, "type") != "DisruptionTarget") return;
        seen = true;
        out->preempt_terminating =
            out->terminating && d.str(c, "status") == "True" && d.str(c, "reason") == "PreemptionByScheduler";
      });
    }
    const JVal* sp = d.get(r, "spec");
    if (!sp) return true;
    out->priority = (int32_t)d.num(*sp, "priority", 0);
    out->preempt_never = d.str(*sp, "preemptionPolicy") == "Never";
    out->node_name = d.str(*sp, "nodeName");
    if (const JVal* ns = d.get(*sp, "nodeSelector")) {
      out->has_node_selector = true;
      out->node_selector = kv_map(d, ns);
    }
    if (const JVal* af = d.get(*sp, "affinity")) {
      if (const JVal* na = d.get(*af, "nodeAffinity")) {
        if (const JVal* rq = d.get(*na, "requiredDuringSchedulingIgnoredDuringExecution")) {
          out->has_required_na = true;
          d.each(d.get(*rq, "nodeSelectorTerms"), [&](const JVal& t) { out->required_na.push_back(ns_term(d, t)); });
        }
        if (const JVal* pf = d.get(*na, "preferredDuringSchedulingIgnoredDuringExecution")) {
          out->has_preferred_na = true;
          d.each(pf, [&](const JVal& t) {
            const JVal* pr = d.get(t, "preference");
            out->preferred_na.push_back({(int32_t)d.num(t, "weight"), pr ? ns_term(d, *pr) : NSTerm{}});
          });
        }
      }
      auto pa = [&](const char* key, bool* has, std::vector<PATerm>* req, std::vector<PATerm>* pref) {
        const JVal* a = d.get(*af, key);
        if (!a) return;
        *has = true;
        d.each(d.get(*a, "requiredDuringSchedulingIgnoredDuringExecution"),
               [&](const JVal& t) { req->push_back(pa_term(d, t, 0)); });
        d.each(d.get(*a, "preferredDuringSchedulingIgnoredDuringExecution"), [&](const JVal& t) {
          const JVal* pt = d.get(t, "podAffinityTerm");
          PATerm x = pt ? pa_term(d, *pt, (int32_t)d.num(t, "weight")) : PATerm{};
          x.weight = (int32_t)d.num(t, "weight");
          pref->push_back(x);
        });
      };
      pa("podAffinity", &out->has_pod_affinity, &out->aff_req, &out->aff_pref);
      pa("podAntiAffinity", &out->has_pod_anti, &out->anti_req, &out->anti_pref);
    }
    d.each(d.get(*sp, "tolerations"), [&](const JVal& t) {
      out->tolerations.push_back({d.str(t, "key"), d.str(t, "operator"), d.str(t, "value"), d.str(t, "effect")});
    });
    bool ok = true;
    d.each(d.get(*sp, "containers"), [&](const JVal& c) {
      Container k;
      ok = ok && container(d, c, &k, err);
      out->containers.push_back(std::move(k));
    });
    d.each(d.get(*sp, "initContainers"), [&](const JVal& c) {
      Container k;
      ok = ok && container(d, c, &k, err);
      out->init_containers.push_back(std::move(k));
    });
    if (!ok) return false;
    auto attach = [&](Container& k) {
      const CStat* found = nullptr;
      for (const CStat& x : cstats)
        if (x.name == k.name) found = &x;  // the last of the name wins (the map's overwrite)
      if (!found || !found->res) return;
      k.has_status = true;
      k.st_req = found->req;
      k.st_alloc = found->alloc;
      out->has_status_res = true;
    };
    for (auto& k : out->containers) attach(k);
    for (auto& k : out->init_containers)
      if (k.sidecar) attach(k);  // only restartable init containers read their status (helpers.go:236-246)
    out->has_status_res = out->has_status_res || out->has_pod_status_res;
    if (const JVal* oh = d.get(*sp, "overhead")) {
      out->has_overhead = true;
      if (!res_list(d, oh, &out->overhead, err)) return false;
    }
    if (const JVal* rs = d.get(*sp, "resources"))
      if (!res_list(d, d.get(*rs, "requests"), &out->pod_requests, err)) return false;
    d.each(d.get(*sp, "topologySpreadConstraints"), [&](const JVal& c) {
      Spread s;
      s.max_skew = (int32_t)d.num(c, "maxSkew");
      s.key = d.str(c, "topologyKey");
      s.when = d.str(c, "whenUnsatisfiable");
      s.sel = label_sel(d, d.get(c, "labelSelector"));
      if (d.present(c, "minDomains")) s.min_domains = (int32_t)d.num(c, "minDomains");
      const std::string ap = d.str(c, "nodeAffinityPolicy"), tp = d.str(c, "nodeTaintsPolicy");
      s.aff_honor = ap.empty() || ap == "Honor";  // common.go:113-114 defaults
      s.taint_honor = tp == "Honor";
      s.match_label_keys = str_list(d, d.get(c, "matchLabelKeys"));
      out->spreads.push_back(std::move(s));
    });
    d.each(d.get(*sp, "volumes"), [&](const JVal& v) {
      if (const JVal* im = d.get(v, "image")) out->image_volumes.push_back(d.str(*im, "reference"));
      // the volume plugins' PreFilter Skip rules: VolumeBinding / VolumeZone / NodeVolumeLimits run for
      // PVC and generic ephemeral volumes (volume_binding.go:350-358, csi.go:239-249) and for in-tree
      // volumes CSI migration translates (csi-translation-lib translate.go:30-38,197-204);
      // VolumeRestrictions for GCE PD / AWS EBS / RBD / iSCSI (volume_restrictions.go:168-197)
      static const char* kPlugged[] = {"persistentVolumeClaim", "ephemeral", "gcePersistentDisk", "awsElasticBlockStore",
                                       "cinder", "azureDisk", "azureFile", "vsphereVolume", "portworxVolume", "rbd",
                                       "iscsi"};
      for (const char* k : kPlugged)
        if (out->unsupported.empty() && d.present(v, k))
          out->unsupported = std::string("volume \"") + d.str(v, "name") + "\" (" + k +
                             ") needs the volume plugins, which run outside the device path";
    });
    bool claims = false;  // DynamicResources PreFilter runs for pods with resource claims (dynamicresources.go:446-479)
    d.each(d.get(*sp, "resourceClaims"), [&](const JVal&) { claims = true; });
    if (claims && out->unsupported.empty())
      out->unsupported = "spec.resourceClaims needs DynamicResources, which runs outside the device path";
    out->scalar_free = pod_scalar_free(*out) ? 1 : 0;
    pod_sign_fragments(d, r, out);
    return true;
  } catch (std::exception& e) {
    *err = e.what();
    return false;
  }
}

// ---- SignPod fragments (kube-scheduler/framework/signers.go; the plugins' SignPod methods) ------------------
// canonical text of a JSON value: object members sorted by name, members that json.Marshal's omitempty would
// leave out of the typed object (null, "", false, empty list / object) dropped
static void canon_json(const JDoc& d, const JVal& v, std::string& o) {
  switch (v.type) {
    case JVal::NUL: o += "null"; return;
    case JVal::BOOL: o += v.b ? "true" : "false"; return;
    case JVal::NUM: o += v.s; return;
    case JVal::STR: o += '"'; o += v.s; o += '"'; return;
    case JVal::ARR: {
      o += '[';
      bool first = true;
      d.each(&v, [&](const JVal& x) {
        if (!first) o += ',';
        first = false;
        canon_json(d, x, o);
      });
      o += ']';
      return;
    }
    case JVal::OBJ: {
      std::vector<const JVal*> kv;
      d.each(&v, [&](const JVal& x) {
        if (x.type == JVal::NUL || (x.type == JVal::STR && x.s.empty()) || (x.type == JVal::BOOL && !x.b) ||
            ((x.type == JVal::ARR || x.type == JVal::OBJ) && x.count == 0))
          return;
        kv.push_back(&x);
      });
      std::sort(kv.begin(), kv.end(), [](const JVal* a, const JVal* b) { return a->key < b->key; });
      o += '{';
      for (size_t i = 0; i < kv.size(); ++i) {
        if (i) o += ',';
        o += '"';
        o += kv[i]->key;
        o += "\":";
        canon_json(d, *kv[i], o);
      }
      o += '}';
      return;
    }
  }
}
static std::string sorted_list(std::vector<std::string> v) {
  std::sort(v.begin(), v.end());
  std::string o = "[";
  for (auto& x : v) o += x + ",";
  return o + "]";
}
static std::string map_text(const JDoc& d, const JVal* m) {  // map[string]string: null when nil
  if (!m) return "null";
  std::vector<std::string> kv;
  d.each(m, [&](const JVal& x) { kv.push_back(x.key + "=" + (x.type == JVal::STR ? x.s : std::string())); });
  std::sort(kv.begin(), kv.end());
  std::string o = "{";
  for (auto& x : kv) o += x + ";";
  return o + "}";
}
// NodeSelectorTermSigner over NodeSelectorRequirementsSigner (signers.go:67-101)
static std::string ns_term_text(const JDoc& d, const JVal* t) {
  auto reqs = [&](const JVal* a) {
    std::vector<std::string> out;
    d.each(a, [&](const JVal& r) {
      std::vector<std::string> vals;
      d.each(d.get(r, "values"), [&](const JVal& x) { vals.push_back(x.s); });
      std::sort(vals.begin(), vals.end());
      std::string t2 = "{key=" + d.str(r, "key") + ";op=" + d.str(r, "operator") + ";values=[";
      for (auto& x : vals) t2 += x + ",";
      out.push_back(t2 + "]}");
    });
    return sorted_list(out);
  };
  return "{exp=" + reqs(t ? d.get(*t, "matchExpressions") : nullptr) + ";fld=" +
         reqs(t ? d.get(*t, "matchFields") : nullptr) + "}";
}
static std::string image_norm(const std::string& n) {  // normalizedImageName (image_locality.go:154-159)
  const size_t c = n.rfind(':'), s = n.rfind('/');
  const long lc = c == std::string::npos ? -1 : (long)c, ls = s == std::string::npos ? -1 : (long)s;
  return lc <= ls ? n + ":latest" : n;
}
static void pod_sign_fragments(const JDoc& d, const JVal& root, PodSpec* out) {
  PodSpec::Sign& f = out->sign;
  const JVal* md = d.get(root, "metadata");
  const JVal* sp = d.get(root, "spec");
  f.labels = map_text(d, md ? d.get(*md, "labels") : nullptr);
  f.sched = sp ? d.str(*sp, "schedulerName") : "";
  f.nsel = map_text(d, sp ? d.get(*sp, "nodeSelector") : nullptr);
  f.na = "null";
  f.tols = f.ports = f.images = f.vols = "[]";
  if (!sp) return;
  {  // TolerationsSigner (:180-189): by (key, value), stable for equal keys
    std::vector<std::pair<std::pair<std::string, std::string>, std::string>> ts;
    d.each(d.get(*sp, "tolerations"), [&](const JVal& t) {
      std::string c;
      canon_json(d, t, c);
      ts.push_back({{d.str(t, "key"), d.str(t, "value")}, c});
    });
    std::stable_sort(ts.begin(), ts.end(), [](auto& a, auto& b) { return a.first < b.first; });
    f.tols = "[";
    for (auto& t : ts) f.tols += t.second + ",";
    f.tols += "]";
  }
  std::vector<int64_t> ports;
  std::vector<std::string> imgs;
  for (const char* key : {"containers", "initContainers"})
    d.each(d.get(*sp, key), [&](const JVal& c) {
      imgs.push_back(image_norm(d.str(c, "image")));
      d.each(d.get(c, "ports"), [&](const JVal& pt) {
        if (d.num(pt, "hostPort") != 0) ports.push_back(d.num(pt, "hostPort"));
      });
      d.each(d.get(c, "restartPolicyRules"), [&](const JVal& r) {  // restartallcontainers.InferForScheduling
        if (d.str(r, "action") == "RestartAllContainers") out->needs_features = true;
      });
    });
  const JVal* hu = d.get(*sp, "hostUsers");  // usernamespaceshostnetwork.InferForScheduling
  if (d.boolean(*sp, "hostNetwork") && hu && hu->type == JVal::BOOL && !hu->b) out->needs_features = true;
  std::sort(ports.begin(), ports.end());  // HostPortsSigner (:50-65)
  ports.erase(std::unique(ports.begin(), ports.end()), ports.end());
  f.ports = "[";
  for (int64_t x : ports) f.ports += std::to_string(x) + ",";
  f.ports += "]";
  std::sort(imgs.begin(), imgs.end());  // ImageLocality.SignPod (image_locality.go:55-67): a sorted set
  imgs.erase(std::unique(imgs.begin(), imgs.end()), imgs.end());
  f.images = "[";
  for (auto& x : imgs) f.images += x + ",";
  f.images += "]";
  std::vector<std::string> vols;  // VolumesSigner (:192-208)
  d.each(d.get(*sp, "volumes"), [&](const JVal& v) {
    if (d.present(v, "configMap") || d.present(v, "secret")) return;
    std::vector<const JVal*> kv;
    d.each(&v, [&](const JVal& x) {
      if (x.key != "name") kv.push_back(&x);
    });
    std::sort(kv.begin(), kv.end(), [](const JVal* a, const JVal* b) { return a->key < b->key; });
    std::string c = "{";
    for (const JVal* x : kv) {  // the VolumeSource: every member but the name (as canon_json, one level up)
      if (x->type == JVal::NUL || (x->type == JVal::STR && x->s.empty()) || (x->type == JVal::BOOL && !x->b) ||
          ((x->type == JVal::ARR || x->type == JVal::OBJ) && x->count == 0))
        continue;
      c += "\"" + x->key + "\":";
      canon_json(d, *x, c);
      c += ",";
    }
    vols.push_back(c + "}");
  });
  f.vols = sorted_list(vols);
  if (const JVal* af = d.get(*sp, "affinity"))  // NodeAffinitySigner (:150-178)
    if (const JVal* na = d.get(*af, "nodeAffinity")) {
      std::vector<std::string> pref, req;
      d.each(d.get(*na, "preferredDuringSchedulingIgnoredDuringExecution"), [&](const JVal& t) {
        pref.push_back("{w=" + std::to_string(d.num(t, "weight")) + ";p=" + ns_term_text(d, d.get(t, "preference")) + "}");
      });
      if (const JVal* rq = d.get(*na, "requiredDuringSchedulingIgnoredDuringExecution"))
        d.each(d.get(*rq, "nodeSelectorTerms"), [&](const JVal& t) { req.push_back(ns_term_text(d, &t)); });
      f.na = "{req=" + sorted_list(req) + ";pref=" + sorted_list(pref) + "}";
    }
  int claims = 0;
  d.each(d.get(*sp, "resourceClaims"), [&](const JVal&) { ++claims; });
  f.claims = claims > 0;
}

bool decode_node(const char* p, size_t n, NodeSpec* out, std::string* err) {
  try {
    JDoc d(p, n);
    const JVal& r = d.root();
    const JVal* md = d.get(r, "metadata");
    if (!md || d.str(*md, "name").empty()) { *err = "node without name"; return false; }
    out->name = d.str(*md, "name");
    out->labels = kv_map(d, d.get(*md, "labels"));
    if (const JVal* sp = d.get(r, "spec")) {
      out->unschedulable = d.boolean(*sp, "unschedulable");
      d.each(d.get(*sp, "taints"), [&](const JVal& t) {
        out->taints.push_back({d.str(t, "key"), d.str(t, "value"), d.str(t, "effect")});
      });
    }
    if (const JVal* st = d.get(r, "status")) {
      if (!res_list(d, d.get(*st, "allocatable"), &out->alloc, err)) return false;
      d.each(d.get(*st, "images"), [&](const JVal& im) {
        out->images.push_back({str_list(d, d.get(im, "names")), d.num(im, "sizeBytes")});
      });
    }
    return true;
  } catch (std::exception& e) {
    *err = e.what();
    return false;
  }
}

bool decode_namespace(const char* p, size_t n, NamespaceSpec* out, std::string* err) {
  try {
    JDoc d(p, n);
    const JVal* md = d.get(d.root(), "metadata");
    if (!md || d.str(*md, "name").empty()) { *err = "namespace without name"; return false; }
    out->name = d.str(*md, "name");
    out->labels = kv_map(d, d.get(*md, "labels"));
    return true;
  } catch (std::exception& e) {
    *err = e.what();
    return false;
  }
}

int obj_kind(const std::string& k) {
  if (k == "Service") return OBJ_SERVICE;
  if (k == "ReplicationController") return OBJ_RC;
  if (k == "ReplicaSet") return OBJ_RS;
  if (k == "StatefulSet") return OBJ_SS;
  return -1;
}

// v1.Service / v1.ReplicationController (spec.selector: map[string]string) and apps/v1 ReplicaSet /
// StatefulSet (spec.selector: *metav1.LabelSelector), the four kinds helper.DefaultSelector lists
bool decode_selector_obj(const char* p, size_t n, SelectorObj* out, std::string* err) {
  try {
    JDoc d(p, n);
    const JVal& r = d.root();
    out->kind = obj_kind(d.str(r, "kind"));
    if (out->kind < 0) { *err = "kind must be Service, ReplicationController, ReplicaSet or StatefulSet"; return false; }
    const JVal* md = d.get(r, "metadata");
    if (!md || d.str(*md, "name").empty()) { *err = "object without name"; return false; }
    out->name = d.str(*md, "name");
    out->ns = d.str(*md, "namespace", "default");
    if (out->ns.empty()) out->ns = "default";  // apiserver defaulting of metadata.namespace
    const JVal* sp = d.get(r, "spec");
    const JVal* sel = sp ? d.get(*sp, "selector") : nullptr;
    if (out->kind == OBJ_SERVICE || out->kind == OBJ_RC) {
      out->sel.present = sel != nullptr;
      out->sel.match = kv_map(d, sel);
    } else {
      out->sel = label_sel(d, sel);
    }
    return true;
  } catch (std::exception& e) {
    *err = e.what();
    return false;
  }
}

// ---- resource requests (component-helpers/resource/helpers.go:151-348) ------------------------
static void add_res(ResVec& a, const ResVec& b) {
  for (const auto& x : b) {
    auto it = std::find_if(a.begin(), a.end(), [&](const ResAmount& r) { return r.name == x.name; });
    if (it == a.end()) a.push_back(x);
    else it->milli += x.milli;
  }
}
static void max_res(ResVec& a, const ResVec& b) {
  for (const auto& x : b) {
    auto it = std::find_if(a.begin(), a.end(), [&](const ResAmount& r) { return r.name == x.name; });
    if (it == a.end()) a.push_back(x);
    else if (x.milli > it->milli) it->milli = x.milli;
  }
}
static bool has_res(const ResVec& a, const std::string& n) {
  return std::any_of(a.begin(), a.end(), [&](const ResAmount& r) { return r.name == n; });
}
static ResVec with_non_missing(const ResVec& req, const ResVec* nm) {
  ResVec out = req;
  if (!nm) return out;
  for (const auto& x : *nm)
    if (!has_res(req, x.name)) add_res(out, {x});
  return out;
}
static bool pod_level_supported(const std::string& n) {
  return n == "cpu" || n == "memory" || n.rfind("hugepages-", 0) == 0;
}

// determineEffectiveRequests (helpers.go:299-304) with max (:494-507): a resize the kubelet reported
// Infeasible counts its actuated and allocated requests only, any other the per-resource maximum of the
// spec, actuated and allocated requests
static ResVec effective_requests(bool infeasible, const ResVec& spec, const ResVec& actuated, const ResVec& alloc) {
  ResVec out = infeasible ? actuated : spec;
  if (!infeasible) max_res(out, actuated);
  max_res(out, alloc);
  return out;
}
static const ResVec& container_requests(const PodSpec& p, const Container& c, bool use_status, ResVec* tmp) {
  if (!use_status || !c.has_status) return c.req;
  *tmp = effective_requests(p.resize_infeasible, c.req, c.st_req, c.st_alloc);
  return *tmp;
}

ResVec pod_requests(const PodSpec& p, const ResVec* non_missing, bool use_status) {
  use_status = use_status && p.has_status_res;
  ResVec reqs, tmp;
  for (const auto& c : p.containers) add_res(reqs, with_non_missing(container_requests(p, c, use_status, &tmp), non_missing));
  ResVec restartable, init;
  for (const auto& c : p.init_containers) {
    ResVec cr = with_non_missing(container_requests(p, c, use_status, &tmp), non_missing);
    if (c.sidecar) {
      add_res(reqs, cr);
      add_res(restartable, cr);
      cr = restartable;
    } else {
      ResVec tmp;
      add_res(tmp, cr);
      add_res(tmp, restartable);
      cr = tmp;
    }
    max_res(init, cr);
  }
  max_res(reqs, init);
  bool pod_level = false;
  for (const auto& r : p.pod_requests) pod_level |= pod_level_supported(r.name);
  if (pod_level) {
    // InPlacePodLevelResourcesVerticalScaling with status.resources set: each pod-level request is the
    // effective one, 0 where that list lacks it (helpers.go:160-179)
    const bool eff = use_status && p.has_pod_status_res;
    const ResVec effr = eff ? effective_requests(p.resize_infeasible, p.pod_requests, p.pod_st_req, p.pod_st_alloc) : ResVec{};
    for (const auto& r : p.pod_requests)
      if (pod_level_supported(r.name)) {
        int64_t v = r.milli;
        if (eff) {
          auto e = std::find_if(effr.begin(), effr.end(), [&](const ResAmount& x) { return x.name == r.name; });
          v = e == effr.end() ? 0 : e->milli;
        }
        auto it = std::find_if(reqs.begin(), reqs.end(), [&](const ResAmount& x) { return x.name == r.name; });
        if (it == reqs.end()) reqs.push_back({r.name, v});
        else it->milli = v;
      }
  }
  if (p.has_overhead) add_res(reqs, p.overhead);
  return reqs;
}

PodResources calc_resources(const PodSpec& p) {  // framework/types.go:1035-1076
  const ResVec requests = pod_requests(p, nullptr, true);
  bool pod_level = false;
  for (const auto& r : p.pod_requests) pod_level |= pod_level_supported(r.name);
  ResVec nm;  // getNonMissingContainerRequests (types.go:1387-1415)
  const int64_t cpu_def = 100, mem_def = 200LL * 1024 * 1024 * 1000;
  if (!pod_level || !has_res(requests, "cpu")) nm.push_back({"cpu", cpu_def});
  if (!pod_level || !has_res(requests, "memory")) nm.push_back({"memory", mem_def});
  const ResVec non0 = nm.empty() ? requests : pod_requests(p, &nm, true);
  PodResources out;
  for (const auto& r : requests) {
    if (r.name == "cpu") out.cpu += r.milli;
    else if (r.name == "memory") out.mem += milli_ceil(r.milli);
    else if (r.name == "ephemeral-storage") out.eph += milli_ceil(r.milli);
    else if (r.name != "pods" && scalar_resource(r.name)) out.scalar.push_back({r.name, milli_ceil(r.milli)});
  }
  for (const auto& r : non0) {
    if (r.name == "cpu") out.nz_cpu = r.milli;
    else if (r.name == "memory") out.nz_mem = milli_ceil(r.milli);
  }
  return out;
}

PodResources calc_fit_request(const PodSpec& p) {  // fit.go:317-325 (SetMaxResource over PodRequests)
  PodResources out;
  for (const auto& r : pod_requests(p, nullptr, false)) {
    if (r.name == "cpu") out.cpu += r.milli;
    else if (r.name == "memory") out.mem += milli_ceil(r.milli);
    else if (r.name == "ephemeral-storage") out.eph += milli_ceil(r.milli);
    else if (r.name != "pods" && scalar_resource(r.name)) out.scalar.push_back({r.name, milli_ceil(r.milli)});
  }
  return out;
}

// api/core/v1/toleration.go:52-112
static bool decimal_integer(const std::string& v) {
  if (v.empty()) return false;
  size_t i = v[0] == '-' ? 1 : 0;
  if (i == v.size()) return false;
  if (v[i] == '0') return v.size() == 1;
  for (; i < v.size(); ++i)
    if (v[i] < '0' || v[i] > '9') return false;
  return true;
}
bool tolerates(const Tol& t, const std::string& key, const std::string& value, const std::string& effect,
               bool cmp_ops) {
  if (!t.effect.empty() && t.effect != effect) return false;
  if (!t.key.empty() && t.key != key) return false;
  if (t.op.empty() || t.op == "Equal") return t.value == value;
  if (t.op == "Exists") return true;
  if ((t.op == "Lt" || t.op == "Gt") && cmp_ops) {
    int64_t a, b;
    if (!decimal_integer(t.value) || !parse_go_int(t.value, &a)) return false;
    if (!decimal_integer(value) || !parse_go_int(value, &b)) return false;
    return t.op == "Lt" ? b < a : b > a;
  }
  return false;
}

// ---- config --------------------------------------------------------------------------------
static const char* kPluginNames[kNumPlugins] = {
    "NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts", "NodeResourcesFit",
    "PodTopologySpread", "InterPodAffinity", "NodeResourcesBalancedAllocation", "ImageLocality"};

Config::Config() {
  static const int64_t w[kNumPlugins] = {0, 0, 3, 2, 0, 1, 2, 2, 1, 1};  // default_plugins.go:35-50
  for (int i = 0; i < kNumPlugins; ++i) {
    enabled[i] = true;
    weight[i] = w[i];
  }
  Spread h, z;  // systemDefaultConstraints (podtopologyspread/plugin.go:46-57), the System defaulting
  h.key = "kubernetes.io/hostname";
  h.when = "ScheduleAnyway";
  h.max_skew = 3;
  z.key = "topology.kubernetes.io/zone";
  z.when = "ScheduleAnyway";
  z.max_skew = 5;
  pts_defaults = {h, z};
}

static int plugin_by_name(const std::string& n) {
  for (int i = 0; i < kNumPlugins; ++i)
    if (n == kPluginNames[i]) return i;
  return -1;
}

// nodeaffinity.newNodeSelectorTerm validity: labels.NewRequirement for matchExpressions
// (apimachinery/pkg/labels/selector.go:210-245), one value + In/NotIn for matchFields
bool valid_ns_term(const NSTerm& t) {
  for (auto& e : t.exprs) {
    if (!valid_label_key(e.key)) return false;
    if (e.op == "In" || e.op == "NotIn") {
      if (e.values.empty()) return false;
    } else if (e.op == "Exists" || e.op == "DoesNotExist") {
      if (!e.values.empty()) return false;
    } else if (e.op == "Gt" || e.op == "Lt") {
      int64_t v;
      if (e.values.size() != 1 || !parse_go_int(e.values[0], &v)) return false;
    } else {
      return false;
    }
    for (auto& v : e.values)
      if (!valid_label_value(v)) return false;
  }
  for (auto& f : t.fields)
    if (f.values.size() != 1 || (f.op != "In" && f.op != "NotIn")) return false;
  return true;
}

bool decode_config(const char* p, size_t n, Config* c, std::string* err) {
  if (!p || n == 0) return true;
  try {
    JDoc d(p, n);
    const JVal& r = d.root();
    if (d.present(r, "percentageOfNodesToScore")) c->pct = (int)d.num(r, "percentageOfNodesToScore");
    if (const JVal* fg = d.get(r, "featureGates")) {
      c->taint_cmp_ops = d.boolean(*fg, "TaintTolerationComparisonOperators");
      const JVal* ob = d.get(*fg, "OpportunisticBatching");  // Beta, on by default (kube_features.go:1674-1676)
      if (ob && ob->type == JVal::BOOL) c->ob_gate = ob->b;
    }
    c->device = (int)d.num(r, "device", 0);
    c->timing_stride = (int)d.num(r, "kernelTimingStride", 0);
    c->loop_timing_stride = (int)d.num(r, "loopTimingStride", 1);
    if (const JVal* pl = d.get(r, "persistentLoop")) c->persistent_loop = pl->type == JVal::BOOL && pl->b;
    c->loop_wg = (int)d.num(r, "loopWorkgroups", 0);
    if (const JVal* rl = d.get(r, "residentLoop")) c->resident_loop = rl->type == JVal::BOOL && rl->b;
    c->loop_unit = (int)d.num(r, "loopUnit", 128) == 256 ? 256 : 128;
    if (const JVal* al = d.get(r, "aggLoop")) c->agg_loop = al->type == JVal::BOOL && al->b;
    c->agg_debug = (int)d.num(r, "aggLoopDebug", 0);
    c->ring_relay_min = (int)d.num(r, "ringRelayMinWorkgroups", 2);
    c->debug_give_up_at = (int)d.num(r, "debugLoopGiveUpAt", -1);
    c->loop_wave_map = (int)d.num(r, "loopWaveMap", 0);
    if (const JVal* ra = d.get(r, "residentAhead")) c->resident_ahead = !(ra->type == JVal::BOOL && !ra->b);
    c->first_chunk = std::max(8, std::min(256, (int)d.num(r, "pipelineFirstChunk", 32)));
    if (c->loop_wave_map < 0 || c->loop_wave_map > 2) c->loop_wave_map = 0;
    if (const JVal* dx = d.get(r, "deviceExchange")) c->dev_exchange = dx->type == JVal::BOOL && dx->b ? 1 : 0;
    c->loop_stamps = d.boolean(r, "loopStamps");
    if (const JVal* ds = d.get(r, "distributed")) {  // node-sharded evaluation
      c->world = (int)d.num(*ds, "worldSize", 1);
      c->rank = (int)d.num(*ds, "rank", 0);
      c->nccl_id = d.str(*ds, "ncclId");
      c->local_group = d.str(*ds, "localGroup");
      if (c->world < 1 || c->world > kMaxShards || c->rank < 0 || c->rank >= c->world) {
        *err = "distributed: worldSize must be in [1, 8] and 0 <= rank < worldSize";
        return false;
      }
      if ((c->world > 1 || !c->nccl_id.empty() || !c->local_group.empty()) &&
          c->nccl_id.empty() == c->local_group.empty()) {
        *err = "distributed: exactly one of ncclId (RCCL) or localGroup (in-process ranks) is required";
        return false;
      }
    }
    bool ok = true;
    d.each(d.get(r, "scoreWeights"), [&](const JVal& v) {
      int id = plugin_by_name(v.key);
      if (id < 0) { ok = false; *err = "unknown plugin " + v.key; return; }
      c->weight[id] = std::strtoll(v.s.c_str(), nullptr, 10);
    });
    d.each(d.get(r, "disabledPlugins"), [&](const JVal& v) {
      int id = plugin_by_name(v.s);
      if (id < 0) { ok = false; *err = "unknown plugin " + v.s; return; }
      c->enabled[id] = false;
    });
    if (!ok) return false;
    auto res_specs = [&](const JVal* a) {
      std::vector<std::pair<std::string, int64_t>> out;
      d.each(a, [&](const JVal& x) {
        int64_t w = d.num(x, "weight", 0);
        out.push_back({d.str(x, "name"), w == 0 ? 1 : w});  // v1 defaulting (defaults.go:218-221)
      });
      return out;
    };
    if (const JVal* f = d.get(r, "nodeResourcesFit")) {
      if (const JVal* ss = d.get(*f, "scoringStrategy")) {
        const std::string t = d.str(*ss, "type", "LeastAllocated");
        if (t == "LeastAllocated") c->fit_strategy = 0;
        else if (t == "MostAllocated") c->fit_strategy = 1;
        else if (t == "RequestedToCapacityRatio") c->fit_strategy = 2;
        else { *err = "unsupported scoring strategy " + t; return false; }
        if (d.present(*ss, "resources")) c->fit_res = res_specs(d.get(*ss, "resources"));
        if (const JVal* rc = d.get(*ss, "requestedToCapacityRatio"))
          d.each(d.get(*rc, "shape"), [&](const JVal& pt) {
            c->rtcr.push_back({d.num(pt, "utilization"), d.num(pt, "score") * 10});  // MaxNodeScore/MaxCustomPriorityScore
          });
      }
      for (auto& s : str_list(d, d.get(*f, "ignoredResources"))) c->ignored_res.insert(s);
      for (auto& s : str_list(d, d.get(*f, "ignoredResourceGroups"))) c->ignored_groups.insert(s);
    }
    if (const JVal* b = d.get(r, "balancedAllocation"))
      if (d.present(*b, "resources")) c->bal_res = res_specs(d.get(*b, "resources"));
    if (const JVal* ipa = d.get(r, "interPodAffinity")) {
      if (d.present(*ipa, "hardPodAffinityWeight")) c->hard_weight = (int32_t)d.num(*ipa, "hardPodAffinityWeight");
      c->ignore_pref_existing = d.boolean(*ipa, "ignorePreferredTermsOfExistingPods");
    }
    {  // PodTopologySpreadArgs (validation_pluginargs.go:102-174; plugin.go:46-57,120-127)
      const JVal* pa = d.get(r, "podTopologySpread");
      const std::string dt = pa ? d.str(*pa, "defaultingType", "System") : "System";  // defaults.go:225-229
      if (dt != "System" && dt != "List") { *err = "podTopologySpread.defaultingType: Unsupported value"; return false; }
      bool bad = false;
      std::vector<Spread> list;
      if (pa)
        d.each(d.get(*pa, "defaultConstraints"), [&](const JVal& x) {
          Spread s;
          s.max_skew = (int32_t)d.num(x, "maxSkew");
          s.key = d.str(x, "topologyKey");
          s.when = d.str(x, "whenUnsatisfiable");
          if (d.present(x, "minDomains")) s.min_domains = (int32_t)d.num(x, "minDomains");
          const std::string ap = d.str(x, "nodeAffinityPolicy"), tp = d.str(x, "nodeTaintsPolicy");
          s.aff_honor = ap.empty() || ap == "Honor";
          s.taint_honor = tp == "Honor";
          if (s.max_skew <= 0 || s.key.empty() || !valid_label_key(s.key) ||
              (s.when != "DoNotSchedule" && s.when != "ScheduleAnyway") || d.present(x, "labelSelector"))
            bad = true;
          for (auto& o : list)
            if (o.key == s.key && o.when == s.when) bad = true;  // validateConstraintNotRepeat
          list.push_back(std::move(s));
        });
      if (bad) { *err = "podTopologySpread.defaultConstraints: invalid constraint"; return false; }
      if (dt == "System" && !list.empty()) {
        *err = "podTopologySpread.defaultingType: Invalid value: \"System\": when .defaultConstraints are not empty";
        return false;
      }
      c->pts_system_defaulted = dt == "System";
      if (!c->pts_system_defaulted) c->pts_defaults = std::move(list);  // System: Config() set them
    }
    if (const JVal* na = d.get(r, "nodeAffinity"))
      if (const JVal* aa = d.get(*na, "addedAffinity")) {
        if (const JVal* rq = d.get(*aa, "requiredDuringSchedulingIgnoredDuringExecution")) {
          c->has_added_required = true;
          d.each(d.get(*rq, "nodeSelectorTerms"), [&](const JVal& t) { c->added_required.push_back(ns_term(d, t)); });
        }
        d.each(d.get(*aa, "preferredDuringSchedulingIgnoredDuringExecution"), [&](const JVal& t) {
          const JVal* pr = d.get(t, "preference");
          c->added_pref.push_back({(int32_t)d.num(t, "weight"), pr ? ns_term(d, *pr) : NSTerm{}});
          c->has_added_pref = true;
        });
      }
    // validation (apis/config/validation/validation_pluginargs.go)
    for (auto& x : c->fit_res)
      if (x.second <= 0 || x.second > 100) { *err = "resource weight of " + x.first + " not in valid range (0, 100]"; return false; }
    std::set<std::string> seen;
    for (auto& x : c->bal_res) {
      if (!seen.insert(x.first).second) { *err = "duplicate resource " + x.first; return false; }
      if (x.second != 1) { *err = "balanced allocation resource weight must be 1"; return false; }
    }
    if (c->hard_weight < 0 || c->hard_weight > 100) { *err = "hardPodAffinityWeight not in [0, 100]"; return false; }
    if (c->fit_strategy == 2) {
      if (c->rtcr.empty()) { *err = "requestedToCapacityRatio shape required"; return false; }
      for (size_t i = 0; i < c->rtcr.size(); ++i) {
        if ((i && c->rtcr[i - 1].first >= c->rtcr[i].first) || c->rtcr[i].first < 0 || c->rtcr[i].first > 100 ||
            c->rtcr[i].second < 0 || c->rtcr[i].second > 100) {
          *err = "invalid requestedToCapacityRatio shape";
          return false;
        }
      }
    }
    for (int i = 0; i < kNumPlugins; ++i)
      if (c->weight[i] < 0) { *err = "negative weight"; return false; }
    // NodeAffinity New(): addedAffinity must parse (node_affinity.go New -> nodeaffinity.NewNodeSelector /
    // NewPreferredSchedulingTerms); empty terms and weight-0 preferred terms are ignored there
    for (auto& t : c->added_required)
      if (!(t.exprs.empty() && t.fields.empty()) && !valid_ns_term(t)) { *err = "invalid addedAffinity"; return false; }
    for (auto& t : c->added_pref)
      if (t.first != 0 && !(t.second.exprs.empty() && t.second.fields.empty()) && !valid_ns_term(t.second)) {
        *err = "invalid addedAffinity";
        return false;
      }
    if (c->pct != 100 && c->pct != 0) { /* accepted; sampling handled by the engine */ }
    return true;
  } catch (std::exception& e) {
    *err = e.what();
    return false;
  }
}

}  // namespace ksg
