// Volcano PodGroup manifest for gang scheduling ([EXT] SyncPodGroup,
// SURVEY C7; RBAC manifests/base/cluster-role.yaml:44-49).
//
// minMember = schedulingPolicy.minAvailable, else the sum of replicas.
// minResources = schedulingPolicy.minResources, else the sum over every
// replica of its containers' requests (limits when no request), so a
// Worker=8 job on MI355X asks the gang scheduler for 8 x amd.com/gpu plus the
// host memory each worker declares -- one 288 GB GPU per worker.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>

#include "core.h"

namespace toa {

// Kubernetes quantity -> base units (cores, bytes, devices)
static double parse_quantity(const std::string& q) {
  if (q.empty()) return 0;
  char* end = nullptr;
  double v = std::strtod(q.c_str(), &end);
  std::string suf = end ? std::string(end) : "";
  static const std::map<std::string, double> mult = {
      {"", 1},        {"m", 1e-3},   {"k", 1e3},          {"M", 1e6},          {"G", 1e9},
      {"T", 1e12},    {"P", 1e15},   {"E", 1e18},         {"Ki", 1024.0},      {"Mi", 1048576.0},
      {"Gi", 1073741824.0}, {"Ti", 1099511627776.0}, {"Pi", 1125899906842624.0}, {"Ei", 1152921504606846976.0},
      {"n", 1e-9},    {"u", 1e-6}};
  auto it = mult.find(suf);
  if (it == mult.end()) {
    // exponent form (1e3) already consumed by strtod
    return v;
  }
  return v * it->second;
}

static std::string format_quantity(const std::string& res, double v) {
  char buf[64];
  if (res == "cpu") {
    double milli = std::round(v * 1000.0);
    if (std::fmod(milli, 1000.0) == 0) snprintf(buf, sizeof buf, "%lld", (long long)(milli / 1000.0));
    else snprintf(buf, sizeof buf, "%lldm", (long long)milli);
    return buf;
  }
  const double Gi = 1073741824.0, Mi = 1048576.0;
  if (v >= Gi && std::fmod(v, Gi) == 0) {
    snprintf(buf, sizeof buf, "%lldGi", (long long)(v / Gi));
    return buf;
  }
  if (v >= Mi && std::fmod(v, Mi) == 0) {
    snprintf(buf, sizeof buf, "%lldMi", (long long)(v / Mi));
    return buf;
  }
  snprintf(buf, sizeof buf, "%lld", (long long)std::llround(v));
  return buf;
}

double pod_resource_request(const Json& replica_spec, const std::string& resource) {
  double total = 0;
  for (const auto& c : replica_spec.path({"template", "spec", "containers"}).items()) {
    const Json* q = c.path({"resources", "requests"}).find(resource);
    if (q == nullptr) q = c.path({"resources", "limits"}).find(resource);
    if (q != nullptr) total += parse_quantity(q->is_string() ? q->str() : q->dump());
  }
  return total;
}

Json gen_podgroup(const Json& job, const Options& opt) {
  const Json& md = job.get("metadata");
  const Json& sp = job.get("spec").get("runPolicy").get("schedulingPolicy");
  const Json& specs = replica_specs(job);
  int64_t total = 0;
  std::map<std::string, double> res;
  for (const auto& kv : specs.fields()) {
    const int64_t n = replicas_of(kv.second);
    total += n;
    for (const auto& c : kv.second.path({"template", "spec", "containers"}).items()) {
      const Json& req = c.path({"resources", "requests"});
      const Json& lim = c.path({"resources", "limits"});
      std::map<std::string, double> per;
      for (const auto& r : lim.fields()) per[r.first] = parse_quantity(r.second.is_string() ? r.second.str() : r.second.dump());
      for (const auto& r : req.fields()) per[r.first] = parse_quantity(r.second.is_string() ? r.second.str() : r.second.dump());
      for (const auto& r : per) res[r.first] += r.second * (double)n;
    }
  }
  Json pg = Json::object();
  pg.set("apiVersion", "scheduling.volcano.sh/v1beta1");
  pg.set("kind", "PodGroup");
  Json pmd = Json::object();
  pmd.set("name", md.get("name").str());
  pmd.set("namespace", md.get("namespace").str("default"));
  Json owners = Json::array();
  owners.push_back(owner_reference(job));
  pmd.set("ownerReferences", owners);
  pg.set("metadata", pmd);
  Json spec = Json::object();
  spec.set("minMember", sp.get("minAvailable").is_null() ? total : sp.get("minAvailable").as_int());
  if (!sp.get("queue").str().empty()) spec.set("queue", sp.get("queue").str());
  if (!sp.get("priorityClass").str().empty()) spec.set("priorityClassName", sp.get("priorityClass").str());
  if (sp.get("minResources").is_object()) {
    spec.set("minResources", sp.get("minResources"));
  } else if (!res.empty()) {
    Json mr = Json::object();
    for (const auto& r : res) mr.set(r.first, format_quantity(r.first, r.second));
    spec.set("minResources", mr);
  }
  pg.set("spec", spec);
  (void)opt;
  return pg;
}

}  // namespace toa
