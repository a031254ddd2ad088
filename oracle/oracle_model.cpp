// oracle_model.cpp -- PARITY ORACLE (test infrastructure; see oracle_model.hpp header).
#include "oracle_model.hpp"

#include <algorithm>
#include <set>
#include <cctype>
#include <cstdio>
#include <climits>

namespace oracle {

// ============================================================================
// resource.Quantity  (apimachinery/pkg/api/resource/quantity.go: parseQuantityString,
// suffix tables in suffix.go; MilliValue = ScaledValue(-3) rounds up)
// ============================================================================
bool parse_quantity_milli(const std::string& s, int64_t* milli) {
  size_t i = 0, n = s.size();
  bool neg = false;
  if (i < n && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  // mantissa as exact integer with a count of fractional digits
  unsigned __int128 mant = 0;
  int frac = 0, ndig = 0;
  bool dot = false;
  for (; i < n; ++i) {
    char c = s[i];
    if (c >= '0' && c <= '9') {
      if (mant < (unsigned __int128)1 << 100) {
        mant = mant * 10 + (unsigned)(c - '0');
        if (dot) ++frac;
      } else if (!dot) {
        return false;  // absurdly large
      }
      ++ndig;
    } else if (c == '.' && !dot) {
      dot = true;
    } else {
      break;
    }
  }
  if (ndig == 0) return false;
  std::string suf = s.substr(i);
  int p2 = 0, p10 = 0;
  static const std::pair<const char*, int> bin[] = {{"Ki", 10}, {"Mi", 20}, {"Gi", 30}, {"Ti", 40}, {"Pi", 50}, {"Ei", 60}};
  static const std::pair<const char*, int> dec[] = {{"n", -9}, {"u", -6}, {"m", -3}, {"", 0}, {"k", 3},
                                                    {"M", 6},  {"G", 9},  {"T", 12}, {"P", 15}, {"E", 18}};
  bool ok = false;
  for (auto& b : bin)
    if (suf == b.first) { p2 = b.second; ok = true; }
  for (auto& d : dec)
    if (suf == d.first) { p10 = d.second; ok = true; }
  if (!ok) {
    if (suf.size() >= 2 && (suf[0] == 'e' || suf[0] == 'E')) {
      int64_t e;
      if (!go_parse_int64(suf.substr(1), &e) || e > 40 || e < -40) return false;
      p10 = (int)e;
    } else {
      return false;
    }
  }
  // value*1000 = mant * 2^p2 * 10^(p10 - frac + 3), rounded up
  unsigned __int128 v = mant;
  const unsigned __int128 lim = (unsigned __int128)1 << 120;
  for (int k = 0; k < p2; ++k) { v <<= 1; if (v > lim) { *milli = neg ? LLONG_MIN : LLONG_MAX; return true; } }
  int e10 = p10 - frac + 3;
  if (e10 >= 0) {
    for (int k = 0; k < e10; ++k) { v *= 10; if (v > lim) { *milli = neg ? LLONG_MIN : LLONG_MAX; return true; } }
  } else {
    unsigned __int128 den = 1;
    for (int k = 0; k < -e10 && den < lim; ++k) den *= 10;
    v = neg ? v / den : (v + den - 1) / den;  // ceil toward +inf
  }
  if (v > (unsigned __int128)LLONG_MAX) v = (unsigned __int128)LLONG_MAX;
  *milli = neg ? -(int64_t)v : (int64_t)v;
  return true;
}

// strconv.ParseInt(s, 10, 64): optional sign, decimal digits, range checked
bool go_parse_int64(const std::string& s, int64_t* out) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  if (i >= s.size()) return false;
  unsigned long long v = 0;
  for (; i < s.size(); ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    unsigned d = s[i] - '0';
    if (v > (ULLONG_MAX - d) / 10) return false;
    v = v * 10 + d;
  }
  if (!neg && v > (unsigned long long)LLONG_MAX) return false;
  if (neg && v > (unsigned long long)LLONG_MAX + 1ull) return false;
  *out = neg ? (int64_t)(0ull - v) : (int64_t)v;
  return true;
}

// ============================================================================
// label validation (apimachinery/pkg/util/validation/validation.go: IsQualifiedName,
// IsValidLabelValue, IsDNS1123Subdomain)
// ============================================================================
static bool qname_part(const std::string& s) {  // ([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9], <=63
  if (s.empty() || s.size() > 63) return false;
  auto an = [](char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); };
  if (!an(s.front()) || !an(s.back())) return false;
  for (char c : s)
    if (!an(c) && c != '-' && c != '_' && c != '.') return false;
  return true;
}
static bool dns1123_subdomain(const std::string& s) {
  if (s.empty() || s.size() > 253) return false;
  size_t start = 0;
  while (true) {
    size_t dot = s.find('.', start);
    std::string lab = s.substr(start, dot == std::string::npos ? std::string::npos : dot - start);
    if (lab.empty()) return false;
    auto lo = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
    if (!lo(lab.front()) || !lo(lab.back())) return false;
    for (char c : lab)
      if (!lo(c) && c != '-') return false;
    if (dot == std::string::npos) break;
    start = dot + 1;
  }
  return true;
}
static bool is_qualified_name(const std::string& k) {
  size_t slash = k.find('/');
  if (slash == std::string::npos) return qname_part(k);
  if (k.find('/', slash + 1) != std::string::npos) return false;
  std::string prefix = k.substr(0, slash), name = k.substr(slash + 1);
  return dns1123_subdomain(prefix) && qname_part(name);
}
static bool is_valid_label_value(const std::string& v) { return v.empty() || qname_part(v); }

// ============================================================================
// labels.Requirement / Selector (apimachinery/pkg/labels/selector.go)
// ============================================================================
bool new_requirement(const std::string& key, Op op, const std::vector<std::string>& vals, Requirement* out) {
  bool ok = is_qualified_name(key);  // validateLabelKey :200
  switch (op) {                       // :203-223
    case Op::In:
    case Op::NotIn:
      if (vals.empty()) ok = false;
      break;
    case Op::Equals:
      if (vals.size() != 1) ok = false;
      break;
    case Op::Exists:
    case Op::DoesNotExist:
      if (!vals.empty()) ok = false;
      break;
    case Op::Gt:
    case Op::Lt: {
      if (vals.size() != 1) ok = false;
      for (auto& v : vals) {
        int64_t x;
        if (!go_parse_int64(v, &x)) ok = false;
      }
      break;
    }
  }
  for (auto& v : vals)  // validateLabelValue :225
    if (!is_valid_label_value(v)) ok = false;
  out->key = key;
  out->op = op;
  out->vals = vals;
  return ok;
}

bool requirement_matches(const Requirement& r, const Labels& ls) {  // selector.go:247-294
  auto it = ls.find(r.key);
  bool exists = it != ls.end();
  auto hasValue = [&](const std::string& v) { return std::find(r.vals.begin(), r.vals.end(), v) != r.vals.end(); };
  switch (r.op) {
    case Op::In:
    case Op::Equals:
      return exists && hasValue(it->second);
    case Op::NotIn:
      return !exists || !hasValue(it->second);
    case Op::Exists:
      return exists;
    case Op::DoesNotExist:
      return !exists;
    case Op::Gt:
    case Op::Lt: {
      if (!exists) return false;
      int64_t lv, rv;
      if (!go_parse_int64(it->second, &lv)) return false;
      if (r.vals.size() != 1) return false;
      if (!go_parse_int64(r.vals[0], &rv)) return false;
      return (r.op == Op::Gt && lv > rv) || (r.op == Op::Lt && lv < rv);
    }
  }
  return false;
}

bool selector_matches(const Selector& s, const Labels& ls) {
  if (s.nothing) return false;  // nothingSelector.Matches :102
  for (auto& r : s.reqs)        // internalSelector.Matches :419-426
    if (!requirement_matches(r, ls)) return false;
  return true;
}

bool label_selector_as_selector(const LabelSelectorSpec& ls, Selector* out) {  // helpers.go:36-71
  *out = Selector{};
  if (!ls.present) { out->nothing = true; return true; }
  if (ls.matchLabels.empty() && ls.matchExpressions.empty()) return true;  // Everything
  for (auto& kv : ls.matchLabels) {
    Requirement r;
    if (!new_requirement(kv.first, Op::Equals, {kv.second}, &r)) return false;
    out->reqs.push_back(r);
  }
  for (auto& e : ls.matchExpressions) {
    Op op;
    if (e.op == "In") op = Op::In;
    else if (e.op == "NotIn") op = Op::NotIn;
    else if (e.op == "Exists") op = Op::Exists;
    else if (e.op == "DoesNotExist") op = Op::DoesNotExist;
    else return false;
    Requirement r;
    if (!new_requirement(e.key, op, e.values, &r)) return false;
    out->reqs.push_back(r);
  }
  std::stable_sort(out->reqs.begin(), out->reqs.end(),
                   [](const Requirement& a, const Requirement& b) { return a.key < b.key; });
  return true;
}

// ============================================================================
// JSON decoding of v1 objects (field names per staging/src/k8s.io/api/core/v1/types.go)
// ============================================================================
static Labels decode_labels(const mj::Value* v) {
  Labels out;
  if (v && v->is_obj())
    for (auto& kv : v->obj)
      if (kv.second.is_str()) out[kv.first] = kv.second.s;
  return out;
}
static std::vector<std::string> decode_strs(const mj::Value* v) {
  std::vector<std::string> out;
  if (v && v->is_arr())
    for (auto& x : v->arr)
      if (x.is_str()) out.push_back(x.s);
  return out;
}
static bool decode_reslist(const mj::Value* v, ResList* out, std::string* err) {
  if (!v || !v->is_obj()) return true;
  for (auto& kv : v->obj) {
    int64_t m = 0;
    std::string txt = kv.second.kind == mj::Value::Number ? kv.second.s : kv.second.s;
    if (!parse_quantity_milli(txt, &m)) {
      *err = "bad quantity " + kv.first + "=" + txt;
      return false;
    }
    (*out)[kv.first] = m;
  }
  return true;
}
LabelSelectorSpec decode_label_selector(const mj::Value* v) {
  LabelSelectorSpec ls;
  if (!v || v->is_null()) return ls;
  ls.present = true;
  if (auto ml = v->has("matchLabels"))
    for (auto& kv : ml->obj)
      if (kv.second.is_str()) ls.matchLabels.push_back({kv.first, kv.second.s});
  if (auto me = v->has("matchExpressions"))
    for (auto& e : me->arr)
      ls.matchExpressions.push_back({e.str("key"), e.str("operator"), decode_strs(e.get("values"))});
  return ls;
}
static std::vector<NSRequirement> decode_ns_reqs(const mj::Value* v) {
  std::vector<NSRequirement> out;
  if (v && v->is_arr())
    for (auto& e : v->arr) out.push_back({e.str("key"), e.str("operator"), decode_strs(e.get("values"))});
  return out;
}
static NodeSelectorTerm decode_term(const mj::Value& v) {
  NodeSelectorTerm t;
  t.matchExpressions = decode_ns_reqs(v.get("matchExpressions"));
  t.matchFields = decode_ns_reqs(v.get("matchFields"));
  return t;
}
static PodAffinityTermSpec decode_pat(const mj::Value& v) {
  PodAffinityTermSpec t;
  t.labelSelector = decode_label_selector(v.get("labelSelector"));
  t.namespaces = decode_strs(v.get("namespaces"));
  t.namespaceSelector = decode_label_selector(v.get("namespaceSelector"));
  t.topologyKey = v.str("topologyKey");
  return t;
}
static bool decode_container(const mj::Value& c, Container* out, std::string* err) {
  out->name = c.str("name");
  out->image = c.str("image");
  if (auto r = c.has("resources"))
    if (!decode_reslist(r->get("requests"), &out->requests, err)) return false;
  if (auto ps = c.has("ports"))
    for (auto& p : ps->arr) {
      ContainerPort cp;
      cp.containerPort = (int32_t)p.i64("containerPort");
      cp.hostPort = (int32_t)p.i64("hostPort");
      cp.hostIP = p.str("hostIP");
      cp.protocol = p.str("protocol");
      out->ports.push_back(cp);
    }
  out->restartAlways = c.str("restartPolicy") == "Always";
  return true;
}

bool decode_node(const mj::Value& v, Node* out, std::string* err) {
  *out = Node{};
  const mj::Value* md = v.has("metadata");
  if (!md) { *err = "node without metadata"; return false; }
  out->name = md->str("name");
  if (out->name.empty()) { *err = "node without name"; return false; }
  out->labels = decode_labels(md->get("labels"));
  if (auto sp = v.has("spec")) {
    out->unschedulable = sp->boolean("unschedulable");
    if (auto ts = sp->has("taints"))
      for (auto& t : ts->arr) out->taints.push_back({t.str("key"), t.str("value"), t.str("effect")});
  }
  if (auto st = v.has("status")) {
    if (!decode_reslist(st->get("allocatable"), &out->allocatable, err)) return false;
    if (auto im = st->has("images"))
      for (auto& i : im->arr) out->images.push_back({decode_strs(i.get("names")), i.i64("sizeBytes")});
  }
  return true;
}

bool decode_namespace(const mj::Value& v, Namespace* out, std::string* err) {
  const mj::Value* md = v.has("metadata");
  if (!md || md->str("name").empty()) { *err = "namespace without name"; return false; }
  out->name = md->str("name");
  out->labels = decode_labels(md->get("labels"));
  return true;
}

// metav1.Time text (RFC 3339 with an optional fraction) -> Unix nanoseconds
static bool rfc3339_ns(const std::string& t, int64_t* out) {
  int Y, M, D, h, m, s, n = 0;
  if (std::sscanf(t.c_str(), "%4d-%2d-%2dT%2d:%2d:%2d%n", &Y, &M, &D, &h, &m, &s, &n) != 6 || n != 19) return false;
  size_t i = 19;
  int64_t frac = 0, scale = 1000000000;
  if (i < t.size() && t[i] == '.') {
    ++i;
    size_t d0 = i;
    while (i < t.size() && isdigit((unsigned char)t[i])) {
      if (scale > 1) { scale /= 10; frac += (t[i] - '0') * scale; }
      ++i;
    }
    if (i == d0) return false;
  }
  int64_t off = 0;
  if (i < t.size() && t[i] == 'Z') ++i;
  else if (i + 6 == t.size() && (t[i] == '+' || t[i] == '-')) {
    int oh, om;
    if (std::sscanf(t.c_str() + i + 1, "%2d:%2d", &oh, &om) != 2) return false;
    off = (t[i] == '+' ? 1 : -1) * (oh * 3600 + om * 60);
    i += 6;
  } else return false;
  if (i != t.size()) return false;
  // days since 1970-01-01 (Howard Hinnant's civil-from-days inverse)
  int64_t y = Y - (M <= 2 ? 1 : 0);
  int64_t era = (y >= 0 ? y : y - 399) / 400;
  int64_t yoe = y - era * 400;
  int64_t mp = (M + 9) % 12;
  int64_t doy = (153 * mp + 2) / 5 + D - 1;
  int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  int64_t days = era * 146097 + doe - 719468;
  *out = (days * 86400 + h * 3600 + m * 60 + s - off) * 1000000000LL + frac;
  return true;
}

TopologySpreadConstraint decode_tsc(const mj::Value& c) {
  TopologySpreadConstraint t;
  t.maxSkew = (int32_t)c.i64("maxSkew");
  t.topologyKey = c.str("topologyKey");
  t.whenUnsatisfiable = c.str("whenUnsatisfiable");
  t.labelSelector = decode_label_selector(c.get("labelSelector"));
  if (c.has("minDomains")) { t.hasMinDomains = true; t.minDomains = (int32_t)c.i64("minDomains"); }
  t.nodeAffinityPolicy = c.str("nodeAffinityPolicy");
  t.nodeTaintsPolicy = c.str("nodeTaintsPolicy");
  t.matchLabelKeys = decode_strs(c.get("matchLabelKeys"));
  return t;
}

bool decode_selector_object(const mj::Value& v, SelectorObject* out, std::string* err) {
  *out = SelectorObject{};
  out->kind = v.str("kind");
  if (out->kind != "Service" && out->kind != "ReplicationController" && out->kind != "ReplicaSet" &&
      out->kind != "StatefulSet") {
    *err = "unsupported kind " + out->kind;
    return false;
  }
  const mj::Value* md = v.has("metadata");
  if (!md || md->str("name").empty()) { *err = "object without name"; return false; }
  out->name = md->str("name");
  out->ns = md->str("namespace", "default");
  if (out->ns.empty()) out->ns = "default";
  const mj::Value* sp = v.has("spec");
  const mj::Value* sel = sp ? sp->has("selector") : nullptr;
  if (out->kind == "Service" || out->kind == "ReplicationController") {
    out->hasMap = sel != nullptr;
    out->map = decode_labels(sel);
  } else {
    out->sel = decode_label_selector(sel);
  }
  return true;
}

bool decode_pod(const mj::Value& v, Pod* out, std::string* err) {
  *out = Pod{};
  const mj::Value* md = v.has("metadata");
  if (!md) { *err = "pod without metadata"; return false; }
  out->name = md->str("name");
  out->ns = md->str("namespace", "default");
  if (out->ns.empty()) out->ns = "default";
  out->uid = md->str("uid");
  if (out->uid.empty()) out->uid = out->ns + "/" + out->name;
  out->labels = decode_labels(md->get("labels"));
  out->terminating = md->has("deletionTimestamp") != nullptr;
  if (auto refs = md->has("ownerReferences"))
    for (auto& r : refs->arr)
      if (!out->hasController && r.boolean("controller")) {
        out->hasController = true;
        out->ownerAPIVersion = r.str("apiVersion");
        out->ownerKind = r.str("kind");
        out->ownerName = r.str("name");
      }
  if (const mj::Value* st = v.has("status")) {
    std::string t = st->str("startTime");
    if (!t.empty()) {
      if (!rfc3339_ns(t, &out->startTimeNs)) { *err = "bad startTime"; return false; }
      out->hasStartTime = true;
    }
    out->nominatedNodeName = st->str("nominatedNodeName");
    if (const mj::Value* cs = st->has("conditions"))
      for (auto& c : cs->arr)
        if (c.str("type") == "DisruptionTarget") {
          out->terminatingByPreemption =
              out->terminating && c.str("status") == "True" && c.str("reason") == "PreemptionByScheduler";
          break;
        }
    if (const mj::Value* cs = st->has("conditions"))
      for (auto& c : cs->arr) out->conditions.push_back({c.str("type"), c.str("reason")});
    auto statuses = [&](const char* key, std::vector<Pod::ContainerStatus>* o) {
      if (const mj::Value* l = st->has(key))
        for (auto& c : l->arr) {
          Pod::ContainerStatus x;
          x.name = c.str("name");
          if (const mj::Value* r = c.has("resources")) {
            x.hasResources = true;
            if (!decode_reslist(r->get("requests"), &x.requests, err)) return false;
          }
          if (!decode_reslist(c.get("allocatedResources"), &x.allocated, err)) return false;
          o->push_back(x);
        }
      return true;
    };
    if (!statuses("containerStatuses", &out->containerStatuses) ||
        !statuses("initContainerStatuses", &out->initContainerStatuses))
      return false;
    if (const mj::Value* r = st->has("resources")) {
      out->hasStatusResources = true;
      if (!decode_reslist(r->get("requests"), &out->statusRequests, err)) return false;
      if (!decode_reslist(st->get("allocatedResources"), &out->statusAllocated, err)) return false;
    }
  }
  const mj::Value* sp = v.has("spec");
  if (!sp) return true;
  out->nodeName = sp->str("nodeName");
  out->priority = (int32_t)sp->i64("priority", 0);
  out->preemptionPolicy = sp->str("preemptionPolicy");
  if (auto ns = sp->has("nodeSelector")) { out->hasNodeSelector = true; out->nodeSelector = decode_labels(ns); }
  if (auto af = sp->has("affinity")) {
    if (auto na = af->has("nodeAffinity")) {
      if (auto rq = na->has("requiredDuringSchedulingIgnoredDuringExecution")) {
        out->hasRequiredNA = true;
        if (auto terms = rq->has("nodeSelectorTerms"))
          for (auto& t : terms->arr) out->requiredNA.push_back(decode_term(t));
      }
      if (auto pf = na->has("preferredDuringSchedulingIgnoredDuringExecution")) {
        out->hasPreferredNA = true;
        for (auto& t : pf->arr) {
          PreferredSchedulingTerm p;
          p.weight = (int32_t)t.i64("weight");
          if (auto pr = t.has("preference")) p.preference = decode_term(*pr);
          out->preferredNA.push_back(p);
        }
      }
    }
    auto decode_pa = [&](const mj::Value* pa, std::vector<PodAffinityTermSpec>* req,
                         std::vector<WeightedPodAffinityTermSpec>* pref) {
      if (auto rq = pa->has("requiredDuringSchedulingIgnoredDuringExecution"))
        for (auto& t : rq->arr) req->push_back(decode_pat(t));
      if (auto pf = pa->has("preferredDuringSchedulingIgnoredDuringExecution"))
        for (auto& t : pf->arr) {
          WeightedPodAffinityTermSpec w;
          w.weight = (int32_t)t.i64("weight");
          if (auto pt = t.has("podAffinityTerm")) w.term = decode_pat(*pt);
          pref->push_back(w);
        }
    };
    if (auto pa = af->has("podAffinity")) { out->hasPodAffinity = true; decode_pa(pa, &out->affReq, &out->affPref); }
    if (auto pa = af->has("podAntiAffinity")) { out->hasPodAntiAffinity = true; decode_pa(pa, &out->antiReq, &out->antiPref); }
  }
  if (auto ts = sp->has("tolerations"))
    for (auto& t : ts->arr) out->tolerations.push_back({t.str("key"), t.str("operator"), t.str("value"), t.str("effect")});
  if (auto cs = sp->has("containers"))
    for (auto& c : cs->arr) {
      Container k;
      if (!decode_container(c, &k, err)) return false;
      out->containers.push_back(k);
    }
  if (auto cs = sp->has("initContainers"))
    for (auto& c : cs->arr) {
      Container k;
      if (!decode_container(c, &k, err)) return false;
      out->initContainers.push_back(k);
    }
  if (auto oh = sp->has("overhead")) {
    out->hasOverhead = true;
    if (!decode_reslist(oh, &out->overhead, err)) return false;
  }
  if (auto rs = sp->has("resources"))
    if (!decode_reslist(rs->get("requests"), &out->podRequests, err)) return false;
  if (auto tsc = sp->has("topologySpreadConstraints"))
    for (auto& c : tsc->arr) out->tsc.push_back(decode_tsc(c));
  if (auto vols = sp->has("volumes"))
    for (auto& vol : vols->arr)
      if (auto im = vol.has("image")) out->imageVolumes.push_back(im->str("reference"));
  sign_fragments(v, out);
  return true;
}

// ============================================================================
// SignPod fragments (kube-scheduler/framework/signers.go; the plugins' SignPod methods)
// ============================================================================
// A canonical text of a JSON value: object keys sorted, null / "" / false / empty members dropped (the
// omitempty fields json.Marshal leaves out of a typed object, so a field written as its zero value and an
// absent one encode alike).
static void canon(const mj::Value& v, std::string& o) {
  switch (v.kind) {
    case mj::Value::Null: o += "null"; return;
    case mj::Value::Bool: o += v.b ? "true" : "false"; return;
    case mj::Value::Number: o += v.s; return;
    case mj::Value::String: o += '"'; o += v.s; o += '"'; return;
    case mj::Value::Array:
      o += '[';
      for (size_t i = 0; i < v.arr.size(); ++i) {
        if (i) o += ',';
        canon(v.arr[i], o);
      }
      o += ']';
      return;
    case mj::Value::Object: {
      std::vector<const std::pair<std::string, mj::Value>*> kv;
      for (auto& m : v.obj) {
        const mj::Value& x = m.second;
        if (x.kind == mj::Value::Null || (x.kind == mj::Value::String && x.s.empty()) ||
            (x.kind == mj::Value::Bool && !x.b) || (x.kind == mj::Value::Array && x.arr.empty()) ||
            (x.kind == mj::Value::Object && x.obj.empty()))
          continue;
        kv.push_back(&m);
      }
      std::sort(kv.begin(), kv.end(), [](auto* a, auto* b) { return a->first < b->first; });
      o += '{';
      for (size_t i = 0; i < kv.size(); ++i) {
        if (i) o += ',';
        o += '"'; o += kv[i]->first; o += "\":";
        canon(kv[i]->second, o);
      }
      o += '}';
      return;
    }
  }
}
static std::string join_sorted(std::vector<std::string> v) {
  std::sort(v.begin(), v.end());
  std::string o = "[";
  for (size_t i = 0; i < v.size(); ++i) o += (i ? "," : "") + v[i];
  return o + "]";
}
static std::string str_map(const mj::Value* m) {  // a map[string]string: null when nil
  if (!m) return "null";
  std::vector<std::string> kv;
  for (auto& e : m->obj) kv.push_back(e.first + "=" + (e.second.kind == mj::Value::String ? e.second.s : std::string()));
  std::sort(kv.begin(), kv.end());
  std::string o = "{";
  for (auto& x : kv) o += x + ";";
  return o + "}";
}
// NodeSelectorRequirementsSigner (signers.go:67-82): each requirement with its values sorted, then the list
static std::string node_reqs_signer(const mj::Value* reqs) {
  std::vector<std::string> out;
  if (reqs)
    for (auto& r : reqs->arr) {
      std::vector<std::string> vals;
      if (auto vs = r.has("values"))
        for (auto& x : vs->arr) vals.push_back(x.s);
      std::sort(vals.begin(), vals.end());
      std::string t = "{key=" + r.str("key") + ";op=" + r.str("operator") + ";values=[";
      for (auto& x : vals) t += x + ",";
      out.push_back(t + "]}");
    }
  return join_sorted(out);
}
static std::string term_signer(const mj::Value* t) {  // NodeSelectorTermSigner (:87-101)
  return "{exp=" + node_reqs_signer(t ? t->has("matchExpressions") : nullptr) +
         ";fld=" + node_reqs_signer(t ? t->has("matchFields") : nullptr) + "}";
}

void sign_fragments(const mj::Value& v, Pod* out) {
  Pod::SignFragments& f = out->sign;
  const mj::Value* sp = v.has("spec");
  const mj::Value* md = v.has("metadata");
  f.labels = str_map(md ? md->has("labels") : nullptr);
  f.schedulerName = sp ? sp->str("schedulerName") : "";
  f.nodeSelector = str_map(sp ? sp->has("nodeSelector") : nullptr);
  if (!sp) {
    f.tolerations = f.hostPorts = f.images = f.volumes = "[]";
    f.nodeAffinity = "null";
    return;
  }
  {  // TolerationsSigner (:180-189): sort.Slice by (key, value) -- an insertion sort, stable, up to 12
    std::vector<std::pair<std::pair<std::string, std::string>, std::string>> ts;
    if (auto tl = sp->has("tolerations"))
      for (auto& t : tl->arr) {
        std::string c;
        canon(t, c);
        ts.push_back({{t.str("key"), t.str("value")}, c});
      }
    std::stable_sort(ts.begin(), ts.end(), [](auto& a, auto& b) { return a.first < b.first; });
    f.tolerations = "[";
    for (auto& t : ts) f.tolerations += t.second + ",";
    f.tolerations += "]";
  }
  std::set<int64_t> ports;  // HostPortsSigner (:50-65): containers then init containers
  std::set<std::string> images;  // ImageLocality.SignPod (image_locality.go:55-67)
  for (const char* key : {"containers", "initContainers"})
    if (auto cs = sp->has(key))
      for (auto& c : cs->arr) {
        images.insert(normalized_image_name(c.str("image")));
        if (auto ps = c.has("ports"))
          for (auto& p : ps->arr)
            if (p.i64("hostPort") != 0) ports.insert(p.i64("hostPort"));
        if (auto rr = c.has("restartPolicyRules"))  // restartallcontainers.InferForScheduling
          for (auto& r : rr->arr)
            if (r.str("action") == "RestartAllContainers") out->needsNodeFeatures = true;
      }
  if (sp->boolean("hostNetwork") && sp->get("hostUsers") && sp->get("hostUsers")->kind == mj::Value::Bool &&
      !sp->boolean("hostUsers", true))
    out->needsNodeFeatures = true;  // usernamespaceshostnetwork.InferForScheduling
  f.hostPorts = "[";
  for (int64_t p : ports) f.hostPorts += std::to_string(p) + ",";
  f.hostPorts += "]";
  f.images = "[";
  for (auto& x : images) f.images += x + ",";
  f.images += "]";
  {  // VolumesSigner (:192-208): every volume but ConfigMap / Secret ones, by its VolumeSource
    std::vector<std::string> vs;
    if (auto vols = sp->has("volumes"))
      for (auto& vol : vols->arr) {
        if (vol.has("configMap") || vol.has("secret")) continue;
        mj::Value src = vol;
        src.obj.erase(std::remove_if(src.obj.begin(), src.obj.end(), [](auto& m) { return m.first == "name"; }),
                      src.obj.end());
        std::string c;
        canon(src, c);
        vs.push_back(c);
      }
    f.volumes = join_sorted(vs);
  }
  f.nodeAffinity = "null";  // NodeAffinitySigner (:150-178): nil without spec.affinity.nodeAffinity
  if (auto af = sp->has("affinity"))
    if (auto na = af->has("nodeAffinity")) {
      std::vector<std::string> pref, req;
      if (auto pf = na->has("preferredDuringSchedulingIgnoredDuringExecution"))
        for (auto& t : pf->arr)
          pref.push_back("{w=" + std::to_string(t.i64("weight")) + ";p=" + term_signer(t.has("preference")) + "}");
      if (auto rq = na->has("requiredDuringSchedulingIgnoredDuringExecution"))
        if (auto terms = rq->has("nodeSelectorTerms"))
          for (auto& t : terms->arr) req.push_back(term_signer(&t));
      f.nodeAffinity = "{req=" + join_sorted(req) + ";pref=" + join_sorted(pref) + "}";
    }
  if (auto rc = sp->has("resourceClaims")) f.hasClaims = !rc->arr.empty();
}

// ============================================================================
// AffinityTerm (kube-scheduler/framework/types.go:387-448)
// ============================================================================
bool AffinityTerm::matches(const Pod& p, const Labels* nsLabels) const {  // :391-396
  static const Labels kEmpty;
  if (namespaces.count(p.ns) || selector_matches(nsSelector, nsLabels ? *nsLabels : kEmpty))
    return selector_matches(selector, p.labels);
  return false;
}

static bool new_affinity_term(const Pod& pod, const PodAffinityTermSpec& t, AffinityTerm* out) {  // :422-448
  if (!label_selector_as_selector(t.labelSelector, &out->selector)) return false;
  out->namespaces.clear();
  if (t.namespaces.empty() && !t.namespaceSelector.present) out->namespaces.insert(pod.ns);
  else out->namespaces.insert(t.namespaces.begin(), t.namespaces.end());
  if (!label_selector_as_selector(t.namespaceSelector, &out->nsSelector)) return false;
  out->topologyKey = t.topologyKey;
  return true;
}

bool new_pod_info(const Pod& p, PodInfo* out) {  // framework/types.go:1183-1226
  out->pod = p;
  out->reqAff.clear(); out->reqAnti.clear(); out->prefAff.clear(); out->prefAnti.clear();
  bool ok = true;
  // GetPodAffinityTerms / GetPodAntiAffinityTerms (kube-scheduler/framework/types.go:454-488)
  auto build = [&](const std::vector<PodAffinityTermSpec>& in, std::vector<AffinityTerm>* o) {
    for (auto& t : in) {
      AffinityTerm a;
      if (!new_affinity_term(p, t, &a)) { ok = false; o->clear(); return; }
      o->push_back(a);
    }
  };
  auto buildw = [&](const std::vector<WeightedPodAffinityTermSpec>& in, std::vector<WeightedAffinityTerm>* o) {
    for (auto& t : in) {
      WeightedAffinityTerm a;
      a.weight = t.weight;
      if (!new_affinity_term(p, t.term, &a.term)) { ok = false; o->clear(); return; }
      o->push_back(a);
    }
  };
  build(p.affReq, &out->reqAff);
  build(p.antiReq, &out->reqAnti);
  buildw(p.affPref, &out->prefAff);
  buildw(p.antiPref, &out->prefAnti);
  out->parseError = !ok;
  out->calc = calculate_resource(p);
  return ok;
}

// ============================================================================
// resources
// ============================================================================
bool is_scalar_resource_name(const std::string& n) {  // scheduler/util/utils.go:200-203 + v1helper
  auto has_prefix = [&](const char* pfx) { return n.rfind(pfx, 0) == 0; };
  bool prefixedNative = n.find("kubernetes.io/") != std::string::npos;
  bool native = n.find('/') == std::string::npos || prefixedNative;
  bool extended = !native && !has_prefix("requests.") && is_qualified_name("requests." + n);
  return extended || has_prefix("hugepages-") || prefixedNative || has_prefix("attachable-volumes-");
}

static void add_list(ResList& a, const ResList& b) {  // helpers.go:474-483
  for (auto& kv : b) a[kv.first] += kv.second;
}
static void max_list(ResList& a, const ResList& b) {  // helpers.go:486-492
  for (auto& kv : b) {
    auto it = a.find(kv.first);
    if (it == a.end() || kv.second > it->second) a[kv.first] = kv.second;
  }
}
static ResList apply_non_missing(const ResList& reqs, const ResList& nonMissing) {  // :334-348
  ResList cp = reqs;
  for (auto& kv : nonMissing)
    if (!reqs.count(kv.first)) cp[kv.first] += kv.second;
  return cp;
}
static bool supported_pod_level(const std::string& n) {  // helpers.go:76-78
  return n == "cpu" || n == "memory" || n.rfind("hugepages-", 0) == 0;
}
bool pod_level_requests_set(const Pod& p) {
  for (auto& kv : p.podRequests)
    if (supported_pod_level(kv.first)) return true;
  return false;
}

static bool is_pod_resize_infeasible(const Pod& p) {  // helpers.go:311-320
  for (auto& c : p.conditions)
    if (c.first == "PodResizePending") return c.second == "Infeasible";
  return false;
}
static ResList max_of(const ResList& a, const ResList& b) {  // max(a, b), helpers.go:494-507
  ResList r = a;
  max_list(r, b);
  return r;
}
// determineEffectiveRequests (helpers.go:299-304)
static ResList determine_effective_requests(const Pod& p, const ResList& spec, const ResList& actuated,
                                            const ResList& allocated) {
  if (is_pod_resize_infeasible(p)) return max_of(actuated, allocated);
  return max_of(max_of(spec, actuated), allocated);
}

ResList pod_requests(const Pod& p, const ResList* nonMissing, bool useStatus, bool skipPodLevel) {  // helpers.go:151-291
  // AggregateContainerRequests (:193-291)
  std::map<std::string, const Pod::ContainerStatus*> containerStatuses;
  if (useStatus) {
    for (auto& cs : p.containerStatuses) containerStatuses[cs.name] = &cs;
    for (auto& cs : p.initContainerStatuses) containerStatuses[cs.name] = &cs;
  }
  ResList reqs;
  for (auto& c : p.containers) {
    ResList cr = c.requests;
    if (useStatus) {
      auto it = containerStatuses.find(c.name);
      if (it != containerStatuses.end() && it->second->hasResources)
        cr = determine_effective_requests(p, c.requests, it->second->requests, it->second->allocated);
    }
    if (nonMissing && !nonMissing->empty()) cr = apply_non_missing(cr, *nonMissing);
    add_list(reqs, cr);
  }
  ResList restartable, initReqs;
  for (auto& c : p.initContainers) {
    ResList cr = c.requests;
    if (useStatus && c.restartAlways) {
      auto it = containerStatuses.find(c.name);
      if (it != containerStatuses.end() && it->second->hasResources)
        cr = determine_effective_requests(p, c.requests, it->second->requests, it->second->allocated);
    }
    if (nonMissing && !nonMissing->empty()) cr = apply_non_missing(cr, *nonMissing);
    if (c.restartAlways) {
      add_list(reqs, cr);
      add_list(restartable, cr);
      cr = restartable;
    } else {
      ResList tmp;
      add_list(tmp, cr);
      add_list(tmp, restartable);
      cr = tmp;
    }
    max_list(initReqs, cr);
  }
  max_list(reqs, initReqs);
  if (!skipPodLevel && pod_level_requests_set(p)) {  // :157-179 (PodLevelResources on by default)
    bool haveEffective = false;
    ResList effectiveReqs;
    if (useStatus && p.hasStatusResources) {  // InPlacePodLevelResourcesVerticalScaling (on by default)
      effectiveReqs = determine_effective_requests(p, p.podRequests, p.statusRequests, p.statusAllocated);
      haveEffective = true;
    }
    for (auto& kv : p.podRequests)
      if (supported_pod_level(kv.first)) {
        reqs[kv.first] = kv.second;
        if (haveEffective) {  // effectiveReqs[name]: the zero Quantity when absent
          auto it = effectiveReqs.find(kv.first);
          reqs[kv.first] = it == effectiveReqs.end() ? 0 : it->second;
        }
      }
  }
  if (p.hasOverhead) add_list(reqs, p.overhead);  // :182-184
  return reqs;
}

PodResource calculate_resource(const Pod& p) {  // framework/types.go:1035-1076 (UseStatusResources: GA gate)
  ResList requests = pod_requests(p, nullptr, true);
  bool podLevelSet = pod_level_requests_set(p);
  ResList nonMissing;  // getNonMissingContainerRequests :1387-1415
  if (!podLevelSet) {
    nonMissing["cpu"] = 100;                       // DefaultMilliCPURequest (util/pod_resources.go:29)
    nonMissing["memory"] = 200LL * 1024 * 1024 * 1000;  // DefaultMemoryRequest, in milli-units
  } else {
    if (!requests.count("cpu")) nonMissing["cpu"] = 100;
    if (!requests.count("memory")) nonMissing["memory"] = 200LL * 1024 * 1024 * 1000;
  }
  ResList non0 = requests;
  if (!nonMissing.empty()) non0 = pod_requests(p, &nonMissing, true);
  PodResource r;
  // Resource.Add (types.go:1270-1291): cpu -> MilliValue, others -> Value
  for (auto& kv : requests) {
    if (kv.first == "cpu") r.res.milliCPU += kv.second;
    else if (kv.first == "memory") r.res.memory += milli_to_value(kv.second);
    else if (kv.first == "pods") r.res.allowedPods += milli_to_value(kv.second);
    else if (kv.first == "ephemeral-storage") r.res.ephemeral += milli_to_value(kv.second);
    else if (is_scalar_resource_name(kv.first)) r.res.scalar[kv.first] += milli_to_value(kv.second);
  }
  r.non0CPU = non0.count("cpu") ? non0["cpu"] : 0;
  r.non0Mem = non0.count("memory") ? milli_to_value(non0["memory"]) : 0;
  return r;
}

// ============================================================================
// tolerations
// ============================================================================
bool g_taint_compare_ops = false;  // TaintTolerationComparisonOperators (kube_features.go:1962, off)

static bool is_decimal_integer(const std::string& v) {  // api/validate/content/decimal_int.go:30-60
  size_t n = v.size(), i = 0;
  if (n == 0) return false;
  if (v[0] == '-') { if (n == 1) return false; i = 1; }
  if (v[i] == '0') return n == 1 && i == 0;
  if (v[i] < '1' || v[i] > '9') return false;
  for (++i; i < n; ++i)
    if (v[i] < '0' || v[i] > '9') return false;
  return true;
}

bool tolerates(const Toleration& t, const Taint& taint) {  // api/core/v1/toleration.go:52-112
  if (!t.effect.empty() && t.effect != taint.effect) return false;
  if (!t.key.empty() && t.key != taint.key) return false;
  if (t.op.empty() || t.op == "Equal") return t.value == taint.value;
  if (t.op == "Exists") return true;
  if (t.op == "Lt" || t.op == "Gt") {
    if (!g_taint_compare_ops) return false;
    int64_t tv, nv;
    if (!is_decimal_integer(t.value) || !go_parse_int64(t.value, &tv)) return false;
    if (!is_decimal_integer(taint.value) || !go_parse_int64(taint.value, &nv)) return false;
    return t.op == "Lt" ? nv < tv : nv > tv;
  }
  return false;
}
bool tolerations_tolerate(const std::vector<Toleration>& ts, const Taint& taint) {  // helpers.go:64-71
  for (auto& t : ts)
    if (tolerates(t, taint)) return true;
  return false;
}
bool find_untolerated_noschedule(const std::vector<Taint>& taints, const std::vector<Toleration>& ts) {
  for (auto& t : taints) {  // helpers.go:79-88 with DoNotScheduleTaintsFilterFunc (helper/taint.go)
    if (t.effect != "NoSchedule" && t.effect != "NoExecute") continue;
    if (!tolerations_tolerate(ts, t)) return true;
  }
  return false;
}

// ============================================================================
// nodeaffinity (component-helpers/scheduling/corev1/nodeaffinity/nodeaffinity.go)
// ============================================================================
ParsedNodeSelectorTerm new_node_selector_term(const NodeSelectorTerm& t) {  // :170-188
  ParsedNodeSelectorTerm out;
  if (!t.matchExpressions.empty()) {  // nodeSelectorRequirementsAsSelector :214-251
    out.hasLabels = true;
    for (auto& e : t.matchExpressions) {
      Op op;
      if (e.op == "In") op = Op::In;
      else if (e.op == "NotIn") op = Op::NotIn;
      else if (e.op == "Exists") op = Op::Exists;
      else if (e.op == "DoesNotExist") op = Op::DoesNotExist;
      else if (e.op == "Gt") op = Op::Gt;
      else if (e.op == "Lt") op = Op::Lt;
      else { out.parseErr = true; continue; }
      Requirement r;
      if (!new_requirement(e.key, op, e.values, &r)) { out.parseErr = true; continue; }
      out.labels.reqs.push_back(r);
    }
    std::stable_sort(out.labels.reqs.begin(), out.labels.reqs.end(),
                     [](const Requirement& a, const Requirement& b) { return a.key < b.key; });
  }
  if (!t.matchFields.empty()) {  // nodeSelectorRequirementsAsFieldSelector :260-293
    out.hasFields = true;
    for (auto& e : t.matchFields) {
      if ((e.op == "In" || e.op == "NotIn") && e.values.size() == 1)
        out.fields.push_back({e.op == "In", {e.key, e.values[0]}});
      else
        out.parseErr = true;
    }
  }
  return out;
}

bool ParsedNodeSelectorTerm::match(const Node& n) const {  // :190-201
  if (parseErr) return false;
  if (hasLabels && !selector_matches(labels, n.labels)) return false;
  if (hasFields && !n.name.empty()) {  // fields = {"metadata.name": name}
    for (auto& f : fields) {
      std::string got = f.second.first == "metadata.name" ? n.name : std::string();
      bool eq = got == f.second.second;
      if (f.first ? !eq : eq) return false;
    }
  }
  return true;
}

bool RequiredNodeAffinity::match(const Node& n) const {  // :323-333
  if (hasLabelSelector && !selector_matches(labelSelector, n.labels)) return false;
  if (hasNodeSelector) {
    for (auto& t : terms)  // LazyErrorNodeSelector.Match :84-103
      if (t.match(n)) return true;
    return false;
  }
  return true;
}

RequiredNodeAffinity get_required_node_affinity(const Pod& p) {  // :306-319
  RequiredNodeAffinity r;
  if (!p.nodeSelector.empty()) {  // labels.SelectorFromSet (no validation)
    r.hasLabelSelector = true;
    for (auto& kv : p.nodeSelector) r.labelSelector.reqs.push_back({kv.first, Op::Equals, {kv.second}});
  }
  if (p.hasRequiredNA) {
    r.hasNodeSelector = true;
    for (auto& t : p.requiredNA) {
      if (t.matchExpressions.empty() && t.matchFields.empty()) continue;  // isEmptyNodeSelectorTerm
      r.terms.push_back(new_node_selector_term(t));
    }
  }
  return r;
}

bool new_node_selector(const std::vector<NodeSelectorTerm>& terms, std::vector<ParsedNodeSelectorTerm>* out) {
  out->clear();  // NewNodeSelector :40-52
  for (auto& t : terms) {
    if (t.matchExpressions.empty() && t.matchFields.empty()) continue;
    auto pt = new_node_selector_term(t);
    if (pt.parseErr) return false;
    out->push_back(pt);
  }
  return true;
}

bool new_preferred_terms(const std::vector<PreferredSchedulingTerm>& in, PreferredTerms* out) {  // :112-135
  out->terms.clear();
  bool ok = true;
  for (auto& t : in) {
    if (t.weight == 0 || (t.preference.matchExpressions.empty() && t.preference.matchFields.empty())) continue;
    auto pt = new_node_selector_term(t.preference);
    if (pt.parseErr) ok = false;
    else out->terms.push_back({t.weight, pt});
  }
  return ok;
}

int64_t preferred_score(const PreferredTerms& t, const Node& n) {  // :139-150
  int64_t s = 0;
  for (auto& kv : t.terms)
    if (kv.second.match(n)) s += kv.first;
  return s;
}

std::string get_zone_key(const Node& n) {  // node/topology/helpers.go:31-58
  auto get = [&](const char* a, const char* b) -> std::string {
    auto it = n.labels.find(a);
    if (it != n.labels.end()) return it->second;
    it = n.labels.find(b);
    return it != n.labels.end() ? it->second : std::string();
  };
  std::string zone = get("failure-domain.beta.kubernetes.io/zone", "topology.kubernetes.io/zone");
  std::string region = get("failure-domain.beta.kubernetes.io/region", "topology.kubernetes.io/region");
  if (region.empty() && zone.empty()) return "";
  return region + std::string(":\0:", 3) + zone;
}

std::string normalized_image_name(const std::string& name) {  // image_locality.go:154-159
  auto colon = name.rfind(':');
  auto slash = name.rfind('/');
  long lc = colon == std::string::npos ? -1 : (long)colon;
  long ls = slash == std::string::npos ? -1 : (long)slash;
  if (lc <= ls) return name + ":latest";
  return name;
}

}  // namespace oracle
