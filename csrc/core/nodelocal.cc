// Single-node xGMI layout for the RCCL ranks of a TFJob / PyTorchJob.
//
// The reference injects cluster-topology env only (TF_CONFIG, MASTER_ADDR /
// RANK / WORLD_SIZE: pkg/controller.v1/tensorflow/tensorflow.go:97-173,
// pytorch/pytorch.go:13-68); its example layout is one `nvidia.com/gpu: 1`
// pod per worker (examples/v1/distribution_strategy/keras-API/
// multi_worker_tfjob.yaml:7-21).  On an MI355X node that layout leaves RCCL
// without its fast path: each pod sees only its own GPU, so there is no
// peer access over xGMI, and every rank believes it is alone on its node
// (LOCAL_WORLD_SIZE = 1).
//
// Node-local mode keeps one pod per replica (per-replica status, restart and
// ExitCode semantics unchanged) and makes the ranks a single-node group:
//
//   * co-location: a required podAffinity on kubernetes.io/hostname to the
//     job's other rank pods (the first pod satisfies its own term), so the
//     scheduler -- or Volcano, which gang-admits the whole PodGroup -- puts
//     every rank on one node; each pod still requests its `amd.com/gpu: 1`,
//     so the node's GPU accounting is unchanged;
//   * peer visibility: hostIPC (dmabuf / IPC handle exchange between the
//     ranks' processes) and the node's /dev/kfd + /dev/dri mounted into the
//     training container, so every rank sees all GPUs of the node and RCCL
//     (and the one-shot IPC all-reduce, parallel/ipc.py) reach peers over
//     xGMI;
//   * env: LOCAL_RANK = the rank's index on the node (= RANK: one node),
//     LOCAL_WORLD_SIZE = the number of ranks on the node, TOA_NODE_LOCAL=1;
//     the trainer binds device TOA_LOCAL_DEVICE when the node agent names
//     the pod's allocated GPU, else LOCAL_RANK (train/dist.py);
//   * the annotation amd.com/gpu-visibility=node, which the local kubelet
//     (localkubelet/kubelet.py) reads to give the pod node-wide visibility.
//
// When: annotation amd.com/node-local "true" (opt in) / "false" (opt out);
// otherwise automatically for a gang-scheduled job whose ranks all request
// exactly one GPU and fit one node (<= Options.gpus_per_node ranks).
// Alternative considered and not taken: packing the ranks into ONE
// `amd.com/gpu: N` pod launched with torchrun -- it collapses Worker=N into a
// single replica and loses the per-replica semantics the CRD promises.
#include "core.h"

namespace toa {

const char* kAnnNodeLocal = "amd.com/node-local";
const char* kAnnGpuVisibility = "amd.com/gpu-visibility";
const char* kLabelNodeLocal = "training.amd.com/node-local";

static bool is_rank_type(const std::string& kind, const std::string& rtype) {
  if (kind == "TFJob") return rtype == "Chief" || rtype == "Master" || rtype == "Worker";
  if (kind == "PyTorchJob") return rtype == "Master" || rtype == "Worker";
  return false;
}

int64_t rank_world(const Json& job) {
  const std::string kind = job_kind(job);
  int64_t world = 0;
  for (const auto& kv : replica_specs(job).fields())
    if (is_rank_type(kind, kv.first) && !kv.second.is_null()) world += replicas_of(kv.second);
  return world;
}

bool node_local(const Json& job, const Options& opt) {
  const std::string kind = job_kind(job);
  if (kind != "TFJob" && kind != "PyTorchJob") return false;
  const std::string mode = lower(job.path({"metadata", "annotations"}).get(kAnnNodeLocal).str());
  if (mode == "false") return false;
  const int64_t world = rank_world(job);
  if (world < 2 || world > opt.gpus_per_node) return false;
  if (mode == "true") return true;
  if (!opt.enable_gang_scheduling) return false;
  for (const auto& kv : replica_specs(job).fields()) {
    if (!is_rank_type(kind, kv.first) || kv.second.is_null()) continue;
    if (pod_resource_request(kv.second, opt.gpu_resource) != 1.0) return false;
  }
  return true;
}

static Json host_path_volume(const std::string& name, const std::string& path) {
  Json v = Json::object();
  v.set("name", name);
  Json hp = Json::object();
  hp.set("path", path);
  v.set("hostPath", hp);
  return v;
}

void apply_node_local(const Json& job, const std::string& rtype, Json& tpl, const Options& opt) {
  const std::string kind = job_kind(job);
  if (!is_rank_type(kind, rtype) || !node_local(job, opt)) return;
  const std::string name = job.get("metadata").get("name").str();
  const KindInfo& ki = kind_info(kind);
  Json& tmd = tpl["metadata"];
  Json labels = tmd.get("labels").is_object() ? tmd.get("labels") : Json::object();
  labels.set(kLabelNodeLocal, "true");
  tmd.set("labels", labels);
  Json ann = tmd.get("annotations").is_object() ? tmd.get("annotations") : Json::object();
  ann.set(kAnnGpuVisibility, "node");
  tmd.set("annotations", ann);

  Json& ps = tpl["spec"];
  ps.set("hostIPC", true);
  // co-locate with the job's other rank pods
  Json sel = Json::object();
  sel.set(kLabelGroupName, labels.get(kLabelGroupName).str("kubeflow.org"));
  sel.set(kLabelJobName, labels.get(kLabelJobName).str(name));
  sel.set(kLabelNodeLocal, "true");
  Json ls = Json::object();
  ls.set("matchLabels", sel);
  Json term = Json::object();
  term.set("labelSelector", ls);
  term.set("topologyKey", "kubernetes.io/hostname");
  Json aff = ps.get("affinity").is_object() ? ps.get("affinity") : Json::object();
  Json pa = aff.get("podAffinity").is_object() ? aff.get("podAffinity") : Json::object();
  Json req = pa.get("requiredDuringSchedulingIgnoredDuringExecution").is_array()
                 ? pa.get("requiredDuringSchedulingIgnoredDuringExecution")
                 : Json::array();
  req.push_back(term);
  pa.set("requiredDuringSchedulingIgnoredDuringExecution", req);
  aff.set("podAffinity", pa);
  ps.set("affinity", aff);

  // the node's GPUs, for peer access over xGMI
  Json vols = ps.get("volumes").is_array() ? ps.get("volumes") : Json::array();
  vols.push_back(host_path_volume("toa-dev-kfd", "/dev/kfd"));
  vols.push_back(host_path_volume("toa-dev-dri", "/dev/dri"));
  ps.set("volumes", vols);
  Json& containers = ps["containers"];
  if (!containers.is_array() || containers.size() == 0) return;
  size_t ci = 0;
  for (size_t i = 0; i < containers.size(); ++i)
    if (containers.at(i).get("name").str() == ki.container) ci = i;
  Json& c = containers.at(ci);
  Json mounts = c.get("volumeMounts").is_array() ? c.get("volumeMounts") : Json::array();
  static const char* const kMounts[2][2] = {{"toa-dev-kfd", "/dev/kfd"}, {"toa-dev-dri", "/dev/dri"}};
  for (const auto& m : kMounts) {
    Json vm = Json::object();
    vm.set("name", m[0]);
    vm.set("mountPath", m[1]);
    mounts.push_back(vm);
  }
  c.set("volumeMounts", mounts);
}

}  // namespace toa
