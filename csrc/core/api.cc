// API constants, defaulting and validation for TFJob / PyTorchJob / MXJob /
// XGBoostJob (kubeflow.org/v1).
//
// Reference: pkg/apis/tensorflow/v1/{constants,defaults,types,util}.go,
// pkg/apis/pytorch/v1/{constants,defaults}.go, pkg/apis/mxnet/v1/...,
// pkg/apis/xgboost/v1/..., pkg/apis/*/validation/validation.go.
// Defaults table: SURVEY Appendix B.
#include <algorithm>
#include <cctype>
#include <stdexcept>

#include <cstdint>

#include "core.h"

namespace toa {

const char* kGroup = "kubeflow.org";
const char* kVersion = "v1";
const char* kApiVersion = "kubeflow.org/v1";
const char* kLabelGroupName = "group-name";
const char* kLabelJobName = "job-name";
const char* kLabelTFJobNameDep = "tf-job-name";
const char* kLabelReplicaType = "replica-type";
const char* kLabelReplicaIndex = "replica-index";
const char* kLabelJobRole = "job-role";
const char* kLabelControllerName = "controller-name";
const char* kGangGroupAnnotation = "scheduling.k8s.io/group-name";
const char* kVolcanoTaskSpec = "volcano.sh/task-spec";

static const std::vector<KindInfo>& kinds() {
  static const std::vector<KindInfo> k = {
      {"TFJob", "tfjobs", "tfjob", "tfReplicaSpecs", "tensorflow", "tfjob-port", 2222, "Never", "Running",
       {"Chief", "Evaluator", "Master", "PS", "Worker"},
       {"PS", "Worker", "Chief", "Master", "Evaluator"}, false, "TFJob", "tfjob-controller"},
      {"PyTorchJob", "pytorchjobs", "pytorchjob", "pytorchReplicaSpecs", "pytorch", "pytorchjob-port", 23456,
       "OnFailure", "None", {"Master", "Worker"}, {"Master", "Worker"}, true, "Job", "pytorchjob-controller"},
      {"MXJob", "mxjobs", "mxjob", "mxReplicaSpecs", "mxnet", "mxjob-port", 9091, "Never", "All",
       {"Scheduler", "Server", "Worker", "TunerTracker", "TunerServer", "Tuner"},
       {"Scheduler", "Server", "Worker"}, false, "MXJob", "mxjob-controller"},
      {"XGBoostJob", "xgboostjobs", "xgboostjob", "xgbReplicaSpecs", "xgboost", "xgboostjob-port", 9999, "Never",
       "All", {"Master", "Worker"}, {"Master", "Worker"}, false, "XGBoostJob", "xgboostjob-controller"},
  };
  return k;
}

const KindInfo& kind_info(const std::string& kind) {
  for (const auto& k : kinds())
    if (k.kind == kind || iequals(k.kind, kind) || k.plural == kind || k.singular == kind) return k;
  throw std::runtime_error("unknown job kind: " + kind);
}

std::vector<std::string> supported_kinds() {
  std::vector<std::string> out;
  for (const auto& k : kinds()) out.push_back(k.kind);
  return out;
}

std::string lower(const std::string& s) {
  std::string o = s;
  std::transform(o.begin(), o.end(), o.begin(), [](unsigned char c) { return (char)std::tolower(c); });
  return o;
}

bool iequals(const std::string& a, const std::string& b) { return lower(a) == lower(b); }

std::string job_kind(const Json& job) {
  std::string k = job.get("kind").str();
  if (!k.empty()) return k;
  // infer from the spec field
  const Json& spec = job.get("spec");
  for (const auto& ki : kinds())
    if (spec.has(ki.specs_field)) return ki.kind;
  return "TFJob";
}

const Json& replica_specs(const Json& job) {
  return job.get("spec").get(kind_info(job_kind(job)).specs_field);
}

int64_t replicas_of(const Json& spec) {
  const Json& r = spec.get("replicas");
  return r.is_null() ? 1 : r.as_int(1);
}

std::string gen_general_name(const std::string& job, const std::string& rt, const std::string& index) {
  std::string n = job + "-" + rt + "-" + index;
  std::replace(n.begin(), n.end(), '/', '-');
  return n;
}

Json gen_labels(const KindInfo& ki, const std::string& job_name) {
  std::string jn = job_name;
  std::replace(jn.begin(), jn.end(), '/', '-');
  Json l = Json::object();
  l.set(kLabelGroupName, kGroup);
  l.set(kLabelJobName, jn);
  if (ki.kind == "TFJob") l.set(kLabelTFJobNameDep, jn);
  l.set(kLabelControllerName, ki.controller_name);
  return l;
}

Json owner_reference(const Json& job) {
  const Json& md = job.get("metadata");
  Json o = Json::object();
  o.set("apiVersion", kApiVersion);
  o.set("kind", job_kind(job));
  o.set("name", md.get("name").str());
  o.set("uid", md.get("uid").str());
  o.set("controller", true);
  o.set("blockOwnerDeletion", true);
  return o;
}

bool is_chief_or_master(const std::string& rtype) { return rtype == "Chief" || rtype == "Master"; }

// port named <kind>-port on the default container of the given replica type
int port_from_job(const Json& job, const std::string& rtype, bool* found) {
  const KindInfo& ki = kind_info(job_kind(job));
  const Json& spec = replica_specs(job).get(rtype);
  for (const auto& c : spec.path({"template", "spec", "containers"}).items()) {
    if (c.get("name").str() != ki.container) continue;
    for (const auto& p : c.get("ports").items()) {
      if (p.get("name").str() == ki.port_name) {
        if (found) *found = true;
        return (int)p.get("containerPort").as_int(ki.port);
      }
    }
  }
  if (found) *found = false;
  return ki.port;
}

// ---------------------------------------------------------------------------
// defaulting
// ---------------------------------------------------------------------------
static void set_default_port(const KindInfo& ki, Json& pod_spec) {
  Json& containers = pod_spec["containers"];
  if (!containers.is_array() || containers.size() == 0) return;
  size_t idx = 0;
  for (size_t i = 0; i < containers.size(); ++i)
    if (containers[i].get("name").str() == ki.container) {
      idx = i;
      break;
    }
  Json& c = containers.at(idx);
  for (const auto& p : c.get("ports").items())
    if (p.get("name").str() == ki.port_name) return;
  Json port = Json::object();
  port.set("name", ki.port_name);
  port.set("containerPort", (int64_t)ki.port);
  c["ports"].push_back(port);
}

Json set_defaults(const Json& job_in) {
  Json job = job_in;
  std::string kind = job_kind(job);
  const KindInfo& ki = kind_info(kind);
  if (job.get("kind").is_null()) job.set("kind", ki.kind);
  if (job.get("apiVersion").is_null()) job.set("apiVersion", kApiVersion);
  Json& spec = job["spec"];
  // legacy flat fields (SDK/YAML examples put cleanPodPolicy etc. at spec root,
  // SURVEY 2.13 quirk 8) are folded into runPolicy.
  static const char* flat[] = {"cleanPodPolicy", "ttlSecondsAfterFinished", "activeDeadlineSeconds", "backoffLimit",
                               "schedulingPolicy"};
  for (const char* f : flat) {
    if (spec.has(f)) {
      if (!spec.get("runPolicy").has(f)) spec["runPolicy"][f] = spec.get(f);
      spec.erase(f);
    }
  }
  Json& rp = spec["runPolicy"];
  if (!rp.is_object()) rp = Json::object();
  if (rp.get("cleanPodPolicy").is_null()) rp.set("cleanPodPolicy", ki.default_clean);
  if (kind == "TFJob" && spec.get("successPolicy").is_null()) spec.set("successPolicy", "");
  if (kind == "MXJob" && spec.get("jobMode").is_null()) spec.set("jobMode", "MXTrain");
  Json& specs = spec[ki.specs_field];
  if (!specs.is_object()) return job;
  // camel-case normalisation of replica-type keys ("ps" -> "PS", "WORKER" -> "Worker")
  for (const auto& canon : ki.camel_types) {
    auto& f = specs.mutable_fields();
    for (auto& kv : f) {
      if (kv.first != canon && iequals(kv.first, canon)) {
        // keep the canonical key if both exist
        bool exists = false;
        for (auto& kv2 : f)
          if (kv2.first == canon) exists = true;
        if (!exists) kv.first = canon;
        break;
      }
    }
  }
  for (auto& kv : specs.mutable_fields()) {
    Json& rs = kv.second;
    if (!rs.is_object()) continue;
    if (rs.get("replicas").is_null()) rs.set("replicas", (int64_t)1);
    if (rs.get("restartPolicy").str().empty()) rs.set("restartPolicy", ki.default_restart);
    if (!ki.port_master_only || kv.first == "Master") {
      Json& ps = rs["template"]["spec"];
      set_default_port(ki, ps);
    }
  }
  return job;
}

// ---------------------------------------------------------------------------
// validation
// ---------------------------------------------------------------------------
static std::string validate_tf_mx(const KindInfo& ki, const Json& specs) {
  const bool tf = ki.kind == "TFJob";
  const std::string pre = tf ? "TFJobSpec is not valid" : "MXJobSpec is not valid";
  if (!specs.is_object()) return pre;
  int found = 0;
  for (const auto& kv : specs.fields()) {
    const std::string& rt = kv.first;
    const Json& v = kv.second;
    const Json& cs = v.path({"template", "spec", "containers"});
    if (!v.is_object() || cs.size() == 0)
      return tf ? pre + ": containers definition expected in " + rt : pre;
    if (tf ? is_chief_or_master(rt) : rt == "Scheduler") found++;
    int named = 0;
    for (const auto& c : cs.items()) {
      if (c.get("image").str().empty()) return tf ? pre + ": Image is undefined in the container of " + rt : pre;
      if (c.get("name").str() == ki.container) named++;
    }
    if (named == 0) return tf ? pre + ": There is no container named " + ki.container + " in " + rt : pre;
  }
  if (found > 1) return tf ? "TFJobSpec is not valid: more than 1 chief/master found" : "more than 1 scheduler found";
  return "";
}

static std::string validate_master_worker(const KindInfo& ki, const Json& specs) {
  const bool pt = ki.kind == "PyTorchJob";
  const std::string sp = pt ? "PyTorchJobSpec" : "XGBoostJobSpec";
  const std::string vp = pt ? "PyTorchJobSpec" : "XGBoostReplicaType";
  if (!specs.is_object()) return sp + " is not valid";
  bool master = false;
  for (const auto& kv : specs.fields()) {
    const std::string& rt = kv.first;
    const Json& v = kv.second;
    const Json& cs = v.path({"template", "spec", "containers"});
    if (!v.is_object() || cs.size() == 0) return sp + " is not valid: containers definition expected in " + rt;
    if (rt != "Master" && rt != "Worker")
      return (pt ? "PyTorchReplicaType is " : "XGBoostReplicaType is ") + rt + " but must be one of [Master Worker]";
    bool present = false;
    for (const auto& c : cs.items()) {
      if (c.get("image").str().empty()) return vp + " is not valid: Image is undefined in the container of " + rt;
      if (c.get("name").str() == ki.container) present = true;
    }
    if (!present) return vp + " is not valid: There is no container named " + ki.container + " in " + rt;
    if (rt == "Master") {
      master = true;
      if (!v.get("replicas").is_null() && v.get("replicas").as_int() != 1)
        return vp + " is not valid: There must be only 1 master replica";
    }
  }
  if (!master) return vp + " is not valid: Master ReplicaSpec must be present";
  return "";
}

std::string validate(const Json& job) {
  const KindInfo* ki = nullptr;
  try {
    ki = &kind_info(job_kind(job));
  } catch (const std::exception& e) {
    return e.what();
  }
  const Json& spec = job.get("spec");
  if (!spec.is_object()) return ki->kind + "Spec is not valid";
  const Json& specs = spec.get(ki->specs_field);
  const std::string err =
      (ki->kind == "TFJob" || ki->kind == "MXJob") ? validate_tf_mx(*ki, specs) : validate_master_worker(*ki, specs);
  if (!err.empty()) return err;
  // elasticPolicy (P9 extension): a Worker group with 1 <= min <= max
  const Json& ep = spec.get("elasticPolicy");
  if (ep.is_null()) return "";
  if (!ep.is_object()) return ki->kind + "Spec is not valid: elasticPolicy must be an object";
  if (!specs.has("Worker")) return ki->kind + "Spec is not valid: elasticPolicy requires a Worker replica spec";
  const int64_t mn = ep.get("minReplicas").as_int(1), mx = ep.get("maxReplicas").as_int(INT64_MAX);
  if (mn < 1) return ki->kind + "Spec is not valid: elasticPolicy.minReplicas must be >= 1";
  if (mx < mn) return ki->kind + "Spec is not valid: elasticPolicy.maxReplicas must be >= minReplicas";
  if (ep.get("maxRestarts").as_int(0) < 0) return ki->kind + "Spec is not valid: elasticPolicy.maxRestarts must be >= 0";
  return "";
}

}  // namespace toa
