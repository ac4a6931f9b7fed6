// tf_operator_amd C++17 operator core -- shared declarations.
//
// The core is PURE and I/O-free: every entry point takes Kubernetes objects
// as JSON values plus the current time, and returns new objects / action
// lists.  The asyncio shell (tf_operator_amd/operator) owns all I/O.
//
// Reference map (paths relative to the reference checkout):
//   api.cc        pkg/apis/{tensorflow,pytorch,mxnet,xgboost}/v1 + validation
//   conditions.cc [EXT] kubeflow/common util/status.go (pinned by
//                 pkg/controller.v1/tensorflow/status_test.go:585-592)
//   envgen.cc     pkg/controller.v1/tensorflow/tensorflow.go, pytorch/pytorch.go,
//                 mxnet/mxnet.go, xgboost/xgboost.go (+ the RCCL/ROCm block)
//   status.cc     tensorflow/status.go:64-220, pytorch/pytorchjob_controller.go:315-393,
//                 mxnet/mxjob_controller.go:328-410, xgboost/xgboostjob_controller.go:324-402
//   reconcile.cc  [EXT] JobController.ReconcileJobs + tensorflow/pod.go ReconcilePods
//   expectations.cc [EXT] controller expectations (client-go semantics)
//   podgroup.cc   [EXT] Volcano PodGroup sync
#pragma once
#include <cmath>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "json.h"

namespace toa {

// ---------------------------------------------------------------------------
// API constants per kind (A1-A7)
// ---------------------------------------------------------------------------
struct KindInfo {
  std::string kind;             // TFJob
  std::string plural;           // tfjobs
  std::string singular;         // tfjob
  std::string specs_field;      // tfReplicaSpecs
  std::string container;        // tensorflow
  std::string port_name;        // tfjob-port
  int port;                     // 2222
  std::string default_restart;  // Never
  std::string default_clean;    // Running
  std::vector<std::string> replica_types;   // canonical names, status-engine order
  std::vector<std::string> camel_types;     // types normalised by defaulting
  bool port_master_only;        // PyTorch: port only added to Master
  std::string reason_prefix;    // TFJob -> TFJobRunning; PyTorchJob -> Job (commonutil reasons)
  std::string controller_name;  // tfjob-controller
};

extern const char* kGroup;         // kubeflow.org
extern const char* kVersion;       // v1
extern const char* kApiVersion;    // kubeflow.org/v1
extern const char* kLabelGroupName;      // group-name
extern const char* kLabelJobName;        // job-name
extern const char* kLabelTFJobNameDep;   // tf-job-name (deprecated)
extern const char* kLabelReplicaType;    // replica-type
extern const char* kLabelReplicaIndex;   // replica-index
extern const char* kLabelJobRole;        // job-role
extern const char* kLabelControllerName; // controller-name
extern const char* kGangGroupAnnotation; // scheduling.k8s.io/group-name
extern const char* kVolcanoTaskSpec;     // volcano.sh/task-spec

const KindInfo& kind_info(const std::string& kind);  // throws on unknown kind
std::vector<std::string> supported_kinds();
std::string lower(const std::string& s);
bool iequals(const std::string& a, const std::string& b);

// defaulting (A2/A4-A6): returns a defaulted copy
Json set_defaults(const Json& job);
// validation (A3/A4-A6): "" when valid, else the reference's error message
std::string validate(const Json& job);

// small helpers used across files
std::string job_kind(const Json& job);
const Json& replica_specs(const Json& job);
int64_t replicas_of(const Json& spec);  // defaulted spec -> replicas (1 if missing)
std::string gen_general_name(const std::string& job, const std::string& rt, const std::string& index);
Json gen_labels(const KindInfo& ki, const std::string& job_name);
Json owner_reference(const Json& job);
int port_from_job(const Json& job, const std::string& rtype, bool* found = nullptr);
bool is_chief_or_master(const std::string& rtype);

// ---------------------------------------------------------------------------
// time (RFC3339, UTC, second precision like metav1.Time)
// ---------------------------------------------------------------------------
std::string rfc3339(double unix_seconds);
double parse_rfc3339(const std::string& s);  // NaN on failure

// ---------------------------------------------------------------------------
// conditions (C5)
// ---------------------------------------------------------------------------
// returns true iff the status changed
bool update_job_conditions(Json& status, const std::string& type, const std::string& reason,
                           const std::string& msg, double now);
bool has_condition(const Json& status, const std::string& type);  // status == True
bool is_succeeded(const Json& status);
bool is_failed(const Json& status);

// ---------------------------------------------------------------------------
// env / cluster spec generation (D5, D7, D8, D9 + ROCm block)
// ---------------------------------------------------------------------------
struct Options {
  std::string cluster_domain;           // CUSTOM_CLUSTER_DOMAIN
  bool enable_gang_scheduling = false;
  std::string gang_scheduler_name = "volcano";
  bool inject_rocm_env = true;          // MASTER_ADDR/RANK/... + NCCL_* for TFJob
  int previous_retry = 0;               // workqueue NumRequeues(job)
  Json nccl_env = Json::object();       // extra NCCL_*/RCCL_* knobs
  bool rccl_defaults = true;            // xGMI-oriented defaults (never override the user's env)
  std::string gpu_resource = "amd.com/gpu";
  int64_t elastic_free_gpus = -1;       // free GPUs for an elastic job (own pods count as free); -1 unknown
  int64_t gpus_per_node = 8;            // node-local layout: at most this many ranks share a node
};
Options options_from_json(const Json& o);

bool tf_is_distributed(const Json& job);
// TF_CONFIG JSON string ("" when not distributed) -- byte-identical to the reference
std::string gen_tf_config(const Json& job, const std::string& rt_lower, int index, const Options& opt);
// environment variables appended to the replica's containers; returns list of
// {"container": name|"*", "name":..., "value":...}
Json gen_env(const Json& job, const std::string& rtype, int index, const Options& opt);
// single-node xGMI layout of the RCCL ranks (nodelocal.cc)
extern const char* kAnnNodeLocal;      // amd.com/node-local: "true" | "false" (default: auto)
extern const char* kAnnGpuVisibility;  // amd.com/gpu-visibility=node on node-local pods
extern const char* kLabelNodeLocal;    // training.amd.com/node-local
// a TFJob PS replica that requests a GPU is an RCCL rank (rank W + p, after
// Chief+Master+Worker): the parameter server on the GPU, parallel/ps_collective.py
bool gpu_ps(const Json& job, const Options& opt);
// Chief+Master+Worker (+ GPU PS) for a TFJob / Master+Worker for a PyTorchJob
int64_t rank_world(const Json& job, const Options& opt);
bool node_local(const Json& job, const Options& opt);
void apply_node_local(const Json& job, const std::string& rtype, Json& pod_template, const Options& opt);
// apply gen_env to a pod template (in place)
void set_cluster_spec(const Json& job, Json& pod_template, const std::string& rtype, int index,
                      const Options& opt);

// ---------------------------------------------------------------------------
// status engines (D4, D6, D8, D9)
// ---------------------------------------------------------------------------
struct StatusResult {
  Json events = Json::array();     // [{type, reason, message}]
  int succeeded = 0, failed = 0;   // metric transitions
};
void update_job_status(const Json& job, const Json& pods, Json& status, double now, StatusResult& out);

// ---------------------------------------------------------------------------
// expectations (C3)
// ---------------------------------------------------------------------------
class Expectations {
 public:
  explicit Expectations(double ttl_seconds = 300.0) : ttl_(ttl_seconds) {}
  void expect_creations(const std::string& key, int n, double now);
  void expect_deletions(const std::string& key, int n, double now);
  void creation_observed(const std::string& key);
  void deletion_observed(const std::string& key);
  bool satisfied(const std::string& key, double now) const;
  void delete_key(const std::string& key);
  std::pair<int64_t, int64_t> get(const std::string& key) const;
  bool exists(const std::string& key) const;

 private:
  struct Rec {
    int64_t add = 0, del = 0;
    double ts = 0;
  };
  double ttl_;
  mutable std::mutex mu_;
  std::map<std::string, Rec> m_;
};
std::string expectation_pods_key(const std::string& job_key, const std::string& rt_lower);
std::string expectation_services_key(const std::string& job_key, const std::string& rt_lower);

// ---------------------------------------------------------------------------
// gang scheduling (C7)
// ---------------------------------------------------------------------------
Json gen_podgroup(const Json& job, const Options& opt);
// per-pod request (limits when no request) of `resource` in a replica spec
double pod_resource_request(const Json& replica_spec, const std::string& resource);

// ---------------------------------------------------------------------------
// elastic worker groups (P9 extension, elastic.cc)
// ---------------------------------------------------------------------------
extern const char* kLabelElasticGeneration;  // training.amd.com/elastic-generation
struct ElasticPlan {
  bool enabled = false;
  bool draining = false;   // old-generation pods still exist: delete them, create nothing
  bool restarted = false;  // a new generation started in this pass
  bool give_up = false;    // maxRestarts exceeded: fail the job
  std::string message;
  Json actions = Json::array();
  Json pods;                      // the current generation's pods
  double requeue_after = NAN;
};
bool is_elastic(const Json& job);
// mutates the defaulted job copy (Worker replicas, generation label/env,
// restartPolicy) and status.elasticStatus
ElasticPlan elastic_prepass(Json& job, const Json& pods, Json& status, double now, const Options& opt);

// ---------------------------------------------------------------------------
// reconcile engine (C1, C2, C4, C6, D1-D3)
// ---------------------------------------------------------------------------
bool is_retryable_exit_code(int code);
Json on_job_created(const Json& job, double now);  // defaults + Created condition
// Full sync of one job.  Result object:
// { "actions": [...], "status": {...}, "status_changed": bool,
//   "requeue_after": seconds|null, "events": [...], "metrics": {...},
//   "expect": [{"key":..., "add":n}], "skipped": reason|null }
Json reconcile(const Json& job, const Json& pods, const Json& services, double now, const Options& opt);

// ControllerRef claiming (claim.cc): {claimed: [objs, adopted ones with our
// controllerRef added], adopt: [names], release: [names], owner_reference}
Json claim_objects(const Json& job, const Json& objs);

}  // namespace toa
