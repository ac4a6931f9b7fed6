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
// ExitCode semantics unchanged) and makes the ranks a single-node group.  It
// is OPT-IN ONLY and has exactly one mechanism for peer-device access:
//
//   annotation amd.com/node-local: "privileged"   ("true" is an alias)
//
//   * co-location: a required podAffinity on kubernetes.io/hostname to the
//     job's other rank pods (the first pod satisfies its own term), so the
//     scheduler -- or Volcano, which gang-admits the whole PodGroup -- puts
//     every rank on one node; each pod still requests its `amd.com/gpu: 1`,
//     so the node's GPU accounting is unchanged;
//   * peer access: the training container runs with
//     securityContext.privileged = true plus the pod's hostIPC.  A hostPath
//     mount of /dev/dri alone does NOT work: a mounted device node is not in
//     the container's device cgroup, so opening a peer GPU fails.  Privileged
//     puts every device of the node in the cgroup, so RCCL (and the one-shot
//     IPC all-reduce, parallel/ipc.py) reach peers over xGMI;
//   * device binding: a privileged container sees every GPU of the node, so
//     LOCAL_RANK cannot name the pod's device -- on a node shared with other
//     jobs rank r would drive GPU r whether or not the device plugin gave it
//     that GPU.  The pod gets the kubelet's pod-resources socket (read-only
//     hostPath) and its own name / namespace (downward API); the trainer asks
//     the kubelet which amd.com/gpu device IDs (PCI addresses) were allocated
//     to THIS pod and binds the HIP device with that PCI address
//     (train/devices.py).  If the answer is unavailable it refuses to start
//     rather than guess;
//   * env: LOCAL_RANK = the rank's index on the node (= RANK: one node),
//     LOCAL_WORLD_SIZE = the number of ranks on the node, TOA_NODE_LOCAL=1,
//     TOA_DEVICE_SOURCE=pod-resources;
//   * the annotation amd.com/gpu-visibility=node, which the local kubelet
//     (localkubelet/kubelet.py) honours only for a privileged container with
//     hostIPC -- the same rule a real node enforces;
//   * RCCL host identity: NCCL_HOSTID from the downward API (spec.nodeName).
//     Every rank pod has its own UTS namespace, so its hostname is the pod
//     name; RCCL (like NCCL) hashes gethostname() + boot_id into hostHash
//     unless NCCL_HOSTID is set, and its P2P / SHM transports refuse a peer
//     with another hostHash ("different node").  Without this value the
//     co-located ranks would form an 8-node communicator over the socket
//     transport -- the degradation this layout exists to prevent.  The
//     required podAffinity puts every rank on one node, so spec.nodeName is
//     the same string in all of them.  A container that sets NCCL_HOSTID
//     itself keeps its own value;
//   * IPC mode: hostPID.  The MI355X hosts support DMA-BUF IPC only
//     (HSA_ENABLE_IPC_MODE_LEGACY=0, kRcclDefaults in envgen.cc; the legacy
//     KFD handles are refused by their driver).  A DMA-BUF IPC handle
//     carries the exporter's PID and fd number, and the importer opens
//     /proc/<pid>/fd/<fd> (ROCm 7.2's libhsa-runtime64: "PID: %jd; fd: %d;
//     /proc/%jd/fd/%d").  So the ranks must see each other's processes:
//     hostPID puts every rank in the node's PID namespace (a per-pod PID
//     namespace would resolve the exporter's PID to nothing or to another
//     process), and the privileged container passes the ptrace-read check
//     that opening another process's fd link makes.  hostIPC stays for the
//     one-shot all-reduce's IPC rendezvous (parallel/ipc.py).  The GPU box
//     refuses unprivileged user namespaces, so
//     scripts/ipc_namespace_probe.py could only run its same-namespace arm
//     there (profiles/r5_ipcns/).
//
// Cost, to be accepted explicitly: privileged pods and hostIPC are rejected by
// the PodSecurity "baseline" and "restricted" levels.  The namespace needs the
// "privileged" level (or an exemption); otherwise pod creation fails and the
// operator records a NodeLocalForbidden Warning event on the job
// (operator/controller.py) instead of leaving it silently Pending.
//
// Requirements (else the layout is not applied and the job runs the
// reference layout): a TFJob / PyTorchJob, 2 <= ranks <= Options.gpus_per_node,
// every rank pod requesting exactly one GPU.  Without the annotation nothing
// changes: no automatic selection.
// Alternative considered and not taken: packing the ranks into ONE
// `amd.com/gpu: N` pod launched with torchrun -- it collapses Worker=N into a
// single replica and loses the per-replica semantics the CRD promises.
#include "core.h"

namespace toa {

const char* kAnnNodeLocal = "amd.com/node-local";
const char* kAnnGpuVisibility = "amd.com/gpu-visibility";
const char* kLabelNodeLocal = "training.amd.com/node-local";
const char* kPodResourcesDir = "/var/lib/kubelet/pod-resources";

// Parameter servers on the GPU.  The reference makes the PS a first-class
// member of the cluster spec (pkg/controller.v1/tensorflow/tensorflow.go:142-173)
// whose variables every worker pushes to and pulls from each step
// (examples/v1/dist-mnist/dist_mnist.py:149-165).  Here a PS replica that
// requests a GPU runs in the SAME RCCL world as the trainers
// (parallel/ps_collective.py: reduce onto the PS during backward, broadcast of
// its shard back), so the operator -- not the payload -- owns that world:
// WORLD_SIZE counts it, its RANK is W + p, and in the node-local layout it is
// co-located and gets the same privileged / hostPID / NCCL_HOSTID treatment,
// so its pushes and pulls take xGMI instead of the socket transport.  A CPU
// PS (no GPU request) stays outside, as before.
bool gpu_ps(const Json& job, const Options& opt) {
  if (job_kind(job) != "TFJob") return false;
  const Json* s = replica_specs(job).find("PS");
  return s && !s->is_null() && replicas_of(*s) > 0 && pod_resource_request(*s, opt.gpu_resource) > 0.0;
}

static bool is_rank_type(const Json& job, const std::string& kind, const std::string& rtype, const Options& opt) {
  if (kind == "TFJob")
    return rtype == "Chief" || rtype == "Master" || rtype == "Worker" || (rtype == "PS" && gpu_ps(job, opt));
  if (kind == "PyTorchJob") return rtype == "Master" || rtype == "Worker";
  return false;
}

int64_t rank_world(const Json& job, const Options& opt) {
  const std::string kind = job_kind(job);
  int64_t world = 0;
  for (const auto& kv : replica_specs(job).fields())
    if (is_rank_type(job, kind, kv.first, opt) && !kv.second.is_null()) world += replicas_of(kv.second);
  return world;
}

bool node_local(const Json& job, const Options& opt) {
  const std::string kind = job_kind(job);
  if (kind != "TFJob" && kind != "PyTorchJob") return false;
  const std::string mode = lower(job.path({"metadata", "annotations"}).get(kAnnNodeLocal).str());
  if (mode != "privileged" && mode != "true") return false;
  const int64_t world = rank_world(job, opt);
  if (world < 2 || world > opt.gpus_per_node) return false;
  for (const auto& kv : replica_specs(job).fields()) {
    if (!is_rank_type(job, kind, kv.first, opt) || kv.second.is_null()) continue;
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
  if (!is_rank_type(job, kind, rtype, opt) || !node_local(job, opt)) return;
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
  ps.set("hostPID", true);  // DMA-BUF IPC handles cross processes by PID (header)
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

  // the kubelet's pod-resources API: which GPU the device plugin gave THIS pod
  Json vols = ps.get("volumes").is_array() ? ps.get("volumes") : Json::array();
  vols.push_back(host_path_volume("toa-pod-resources", kPodResourcesDir));
  ps.set("volumes", vols);
  Json& containers = ps["containers"];
  if (!containers.is_array() || containers.size() == 0) return;
  size_t ci = 0;
  for (size_t i = 0; i < containers.size(); ++i)
    if (containers.at(i).get("name").str() == ki.container) ci = i;
  Json& c = containers.at(ci);
  Json mounts = c.get("volumeMounts").is_array() ? c.get("volumeMounts") : Json::array();
  Json vm = Json::object();
  vm.set("name", "toa-pod-resources");
  vm.set("mountPath", kPodResourcesDir);
  vm.set("readOnly", true);
  mounts.push_back(vm);
  c.set("volumeMounts", mounts);
  // every GPU of the node in the container's device cgroup (peer access)
  Json sc = c.get("securityContext").is_object() ? c.get("securityContext") : Json::object();
  sc.set("privileged", true);
  c.set("securityContext", sc);
  // the pod's own identity, for the pod-resources lookup; the node's name as
  // RCCL's host identity (header: one hostHash for every rank of the node)
  Json env = c.get("env").is_array() ? c.get("env") : Json::array();
  static const char* const kDownward[3][2] = {{"TOA_POD_NAME", "metadata.name"},
                                              {"TOA_POD_NAMESPACE", "metadata.namespace"},
                                              {"NCCL_HOSTID", "spec.nodeName"}};
  for (const auto& d : kDownward) {
    bool have = false;
    for (size_t i = 0; i < env.size(); ++i) have = have || env.at(i).get("name").str() == d[0];
    if (have) continue;
    Json fr = Json::object();
    fr.set("fieldPath", d[1]);
    Json vf = Json::object();
    vf.set("fieldRef", fr);
    Json e = Json::object();
    e.set("name", d[0]);
    e.set("valueFrom", vf);
    env.push_back(e);
  }
  c.set("env", env);
}

}  // namespace toa
