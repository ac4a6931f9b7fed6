// Cluster-spec / rendezvous environment generation for every replica.
//
// * TFJob: TF_CONFIG, byte-identical to the reference
//   (pkg/controller.v1/tensorflow/tensorflow.go:97-173, pinned by
//   pod_test.go:230-281 and tensorflow_test.go:23-45), only on the
//   `tensorflow` container and only for distributed jobs (pod.go:261-319);
//   PLUS the ROCm/RCCL block consumed by the PyTorch-ROCm trainer:
//   MASTER_ADDR/MASTER_PORT (rank-0 = Chief, else Master, else Worker-0),
//   WORLD_SIZE (= Chief+Master+Worker, plus the PS replicas when they request
//   a GPU -- nodelocal.cc gpu_ps -- as ranks W..W+P-1; a CPU PS and the
//   Evaluator stay outside the RCCL world), RANK, LOCAL_RANK/LOCAL_WORLD_SIZE
//   (one GPU per pod; in the
//   node-local layout -- nodelocal.cc -- the rank's index on the one node
//   and the node's rank count),
//   TOA_ROLE / TOA_PS_HOSTS for parameter-server mode, NCCL_* knobs.
// * PyTorchJob: pytorch/pytorch.go:13-96 (every container).
// * MXJob: mxnet/mxnet.go:55-233 (MX_CONFIG + DMLC_* + BytePS id).
// * XGBoostJob: xgboost/xgboost.go:14-135.
#include <algorithm>
#include <cstdlib>

#include "core.h"

namespace toa {

Options options_from_json(const Json& o) {
  Options opt;
  if (!o.is_object()) return opt;
  opt.cluster_domain = o.get("cluster_domain").str();
  opt.enable_gang_scheduling = o.get("enable_gang_scheduling").as_bool(false);
  opt.gang_scheduler_name = o.get("gang_scheduler_name").str("volcano");
  if (o.has("inject_rocm_env")) opt.inject_rocm_env = o.get("inject_rocm_env").as_bool(true);
  opt.previous_retry = (int)o.get("previous_retry").as_int(0);
  if (o.get("nccl_env").is_object()) opt.nccl_env = o.get("nccl_env");
  if (o.has("rccl_defaults")) opt.rccl_defaults = o.get("rccl_defaults").as_bool(true);
  opt.gpu_resource = o.get("gpu_resource").str("amd.com/gpu");
  opt.elastic_free_gpus = o.get("elastic_free_gpus").as_int(-1);
  opt.gpus_per_node = o.get("gpus_per_node").as_int(8);
  return opt;
}

bool tf_is_distributed(const Json& job) {
  const Json& specs = replica_specs(job);
  int64_t n = 0;
  for (const char* t : {"Chief", "Evaluator", "Master", "PS", "Worker"}) {
    const Json* s = specs.find(t);
    if (!s || s->is_null()) continue;
    n += s->get("replicas").is_null() ? 1 : s->get("replicas").as_int();
  }
  return n != 1;
}

static std::string svc_endpoint(const Json& job, const std::string& rt_lower, int i, int port, const Options& opt) {
  const Json& md = job.get("metadata");
  std::string host = gen_general_name(md.get("name").str(), rt_lower, std::to_string(i));
  std::string ns = md.get("namespace").str("default");
  std::string svc = host + "." + ns + ".svc";
  if (!opt.cluster_domain.empty()) svc += "." + opt.cluster_domain;
  return svc + ":" + std::to_string(port);
}

// cluster: rt_lower -> [endpoints], as an object with sorted keys (Go map order)
static Json tf_cluster_spec(const Json& job, const Options& opt) {
  std::vector<std::pair<std::string, Json>> entries;
  for (const auto& kv : replica_specs(job).fields()) {
    std::string rt = lower(kv.first);
    int port = port_from_job(job, kv.first);
    int64_t n = replicas_of(kv.second);
    Json list = Json::array();
    for (int64_t i = 0; i < n; ++i) list.push_back(svc_endpoint(job, rt, (int)i, port, opt));
    entries.emplace_back(rt, list);
  }
  std::sort(entries.begin(), entries.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  Json c = Json::object();
  for (auto& e : entries) c.set(e.first, e.second);
  return c;
}

std::string gen_tf_config(const Json& job, const std::string& rt_lower, int index, const Options& opt) {
  Json cluster = tf_cluster_spec(job, opt);
  Json task = Json::object();
  task.set("type", rt_lower);
  task.set("index", (int64_t)index);
  Json cfg = Json::object();
  if (job.get("spec").get("enableDynamicWorker").as_bool(false)) {
    // SparseTFConfig {sparseCluster:{worker:{idx:addr}, ps:[...]}, task}
    Json workers = Json::object();
    Json ps = Json::array();
    if (rt_lower == "ps") {
      const Json& l = cluster.get("ps");
      if ((size_t)index < l.size()) ps.push_back(l[index]);
    } else if (rt_lower == "worker") {
      const Json& l = cluster.get("worker");
      if ((size_t)index < l.size()) workers.set(std::to_string(index), l[index]);
      ps = cluster.get("ps");  // Go: nil slice -> null when there is no PS
    }
    Json sc = Json::object();
    sc.set("worker", workers);
    sc.set("ps", ps);
    cfg.set("sparseCluster", sc);
    cfg.set("task", task);
  } else {
    cfg.set("cluster", cluster);
    cfg.set("task", task);
    cfg.set("environment", "cloud");
  }
  return cfg.dump(false);
}

static void add_env(Json& out, const std::string& container, const std::string& name, const std::string& value) {
  Json e = Json::object();
  e.set("container", container);
  e.set("name", name);
  e.set("value", value);
  out.push_back(e);
}

// Defaults for RCCL over xGMI on an MI355X node, appended only when neither
// --nccl-env nor the container itself sets the variable (set_cluster_spec
// skips entries marked "default" that the container already defines):
//  * TORCH_NCCL_HIGH_PRIORITY: the bucketed reduce-scatter / all-gather run on
//    high-priority HIP streams, so they are not queued behind the backward
//    GEMMs they are meant to overlap;
//  * TORCH_NCCL_AVOID_RECORD_STREAMS: async collectives keep their inputs
//    alive by reference instead of recordStream (no delayed frees of the
//    flat gradient buckets in the caching allocator);
//  * HSA_ENABLE_IPC_MODE_LEGACY=0: dmabuf IPC, which RCCL's P2P transport and
//    CUDA-tensor sharing between processes need on ROCm 7 drivers.
static const char* const kRcclDefaults[][2] = {
    {"TORCH_NCCL_HIGH_PRIORITY", "1"},
    {"TORCH_NCCL_AVOID_RECORD_STREAMS", "1"},
    {"HSA_ENABLE_IPC_MODE_LEGACY", "0"},
};

static void add_default_env(Json& out, const std::string& container, const std::string& name,
                            const std::string& value) {
  Json e = Json::object();
  e.set("container", container);
  e.set("name", name);
  e.set("value", value);
  e.set("default", true);
  out.push_back(e);
}

static int64_t spec_replicas(const Json& job, const std::string& rt) {
  const Json* s = replica_specs(job).find(rt);
  return (s && !s->is_null()) ? replicas_of(*s) : 0;
}

static void rocm_block(const Json& job, const std::string& rtype, int index, const Options& opt,
                       const std::string& container, Json& out) {
  const Json& md = job.get("metadata");
  const std::string name = md.get("name").str();
  add_env(out, container, "TOA_JOB_NAME", name);
  add_env(out, container, "TOA_JOB_KIND", job_kind(job));
  add_env(out, container, "TOA_JOB_NAMESPACE", md.get("namespace").str("default"));
  add_env(out, container, "TOA_REPLICA_TYPE", lower(rtype));
  add_env(out, container, "TOA_REPLICA_INDEX", std::to_string(index));
  for (const auto& kv : opt.nccl_env.fields()) add_env(out, container, kv.first, kv.second.is_string() ? kv.second.str() : kv.second.dump());
  if (opt.rccl_defaults)
    for (const auto& d : kRcclDefaults)
      if (!opt.nccl_env.has(d[0])) add_default_env(out, container, d[0], d[1]);
  const Json& ann = md.get("annotations");
  if (ann.has("amd.com/checkpoint-dir")) add_env(out, container, "TOA_CHECKPOINT_DIR", ann.get("amd.com/checkpoint-dir").str());
}

Json gen_env(const Json& job, const std::string& rtype, int index, const Options& opt) {
  const std::string kind = job_kind(job);
  const KindInfo& ki = kind_info(kind);
  const std::string rt = lower(rtype);
  Json out = Json::array();
  if (kind == "TFJob") {
    const std::string c = ki.container;
    if (tf_is_distributed(job)) add_env(out, c, "TF_CONFIG", gen_tf_config(job, rt, index, opt));
    if (!opt.inject_rocm_env) return out;
    // --- ROCm / RCCL rendezvous block ---
    int64_t n_chief = spec_replicas(job, "Chief"), n_master = spec_replicas(job, "Master");
    int64_t n_worker = spec_replicas(job, "Worker"), n_ps = spec_replicas(job, "PS");
    std::string r0 = n_chief > 0 ? "Chief" : (n_master > 0 ? "Master" : "Worker");
    const int64_t trainers = n_chief + n_master + n_worker;
    const bool ps_ranks = gpu_ps(job, opt);
    int64_t world = trainers + (ps_ranks ? n_ps : 0);
    std::string role = rt;
    rocm_block(job, rtype, index, opt, c, out);
    if (world > 0) {
      std::string ep = svc_endpoint(job, lower(r0), 0, port_from_job(job, r0), opt);
      std::string host = ep.substr(0, ep.rfind(':'));
      add_env(out, c, "MASTER_ADDR", host);
      add_env(out, c, "MASTER_PORT", std::to_string(port_from_job(job, r0)));
      add_env(out, c, "WORLD_SIZE", std::to_string(world));
    }
    int64_t rank = -1;
    if (rtype == "Chief") rank = index;
    else if (rtype == "Master") rank = n_chief + index;
    else if (rtype == "Worker") rank = n_chief + n_master + index;
    else if (rtype == "PS" && ps_ranks) rank = trainers + index;
    if (rank >= 0) {
      const bool nl = node_local(job, opt);
      add_env(out, c, "RANK", std::to_string(rank));
      add_env(out, c, "LOCAL_RANK", nl ? std::to_string(rank) : "0");
      add_env(out, c, "LOCAL_WORLD_SIZE", nl ? std::to_string(world) : "1");
      if (nl) {
        add_env(out, c, "TOA_NODE_LOCAL", "1");
        add_env(out, c, "TOA_DEVICE_SOURCE", "pod-resources");
      }
    }
    add_env(out, c, "TOA_ROLE", role);
    if (n_ps > 0) {
      // the trainer checks the world against these (ps_collective.ps_world_env)
      add_env(out, c, "TOA_PS_IN_WORLD", ps_ranks ? "1" : "0");
      add_env(out, c, "TOA_NUM_TRAINERS", std::to_string(trainers));
      std::string hosts;
      int port = port_from_job(job, "PS");
      for (int64_t i = 0; i < n_ps; ++i) {
        if (i) hosts += ",";
        hosts += svc_endpoint(job, "ps", (int)i, port, opt);
      }
      add_env(out, c, "TOA_PS_HOSTS", hosts);
    }
    return out;
  }
  if (kind == "PyTorchJob") {
    int64_t total = 0;
    for (const auto& kv : replica_specs(job).fields()) total += replicas_of(kv.second);
    int port = port_from_job(job, "Master");
    std::string addr = gen_general_name(job.get("metadata").get("name").str(), "master", "0");
    int64_t rank = index;
    if (rt == "master") addr = "localhost";
    else rank = index + 1;
    add_env(out, "*", "MASTER_PORT", std::to_string(port));
    add_env(out, "*", "MASTER_ADDR", addr);
    add_env(out, "*", "WORLD_SIZE", std::to_string(total));
    add_env(out, "*", "RANK", std::to_string(rank));
    add_env(out, "*", "PYTHONUNBUFFERED", "0");
    if (opt.inject_rocm_env) {
      const bool nl = node_local(job, opt);
      add_env(out, "*", "LOCAL_RANK", nl ? std::to_string(rank) : "0");
      add_env(out, "*", "LOCAL_WORLD_SIZE", nl ? std::to_string(total) : "1");
      if (nl) {
        add_env(out, "*", "TOA_NODE_LOCAL", "1");
        add_env(out, "*", "TOA_DEVICE_SOURCE", "pod-resources");
      }
      rocm_block(job, rtype, index, opt, "*", out);
    }
    return out;
  }
  if (kind == "MXJob") {
    // MX_CONFIG {cluster: {rt:[{url,port}]}, labels: {rt: annotation}, task: {type, index}}
    std::vector<std::pair<std::string, Json>> cl, lb;
    for (const auto& kv : replica_specs(job).fields()) {
      std::string r = lower(kv.first);
      int port = port_from_job(job, kv.first);
      Json list = Json::array();
      for (int64_t i = 0; i < replicas_of(kv.second); ++i) {
        Json up = Json::object();
        up.set("url", gen_general_name(job.get("metadata").get("name").str(), r, std::to_string(i)));
        up.set("port", (int64_t)port);
        list.push_back(up);
      }
      cl.emplace_back(r, list);
      lb.emplace_back(r, kv.second.path({"template", "metadata", "annotations"}).get("tuner-server-key").str());
    }
    auto by_key = [](const auto& a, const auto& b) { return a.first < b.first; };
    std::sort(cl.begin(), cl.end(), by_key);
    std::sort(lb.begin(), lb.end(), by_key);
    Json cluster = Json::object(), labels = Json::object();
    for (auto& e : cl) cluster.set(e.first, e.second);
    for (auto& e : lb) labels.set(e.first, e.second);
    Json task = Json::object();
    task.set("type", rt);
    task.set("index", (int64_t)index);
    Json cfg = Json::object();
    cfg.set("cluster", cluster);
    cfg.set("labels", labels);
    cfg.set("task", task);
    const Json& sched = cluster.get("scheduler");
    std::string root_port = "0", root_uri;
    if (sched.size() > 0) {
      root_port = std::to_string(sched[0].get("port").as_int());
      root_uri = sched[0].get("url").str();
    }
    add_env(out, "*", "MX_CONFIG", cfg.dump(false));
    add_env(out, "*", "DMLC_PS_ROOT_PORT", root_port);
    add_env(out, "*", "DMLC_PS_ROOT_URI", root_uri);
    add_env(out, "*", "DMLC_NUM_SERVER", std::to_string(cluster.get("server").size()));
    add_env(out, "*", "DMLC_NUM_WORKER", std::to_string(cluster.get("worker").size()));
    add_env(out, "*", "DMLC_ROLE", rt);
    add_env(out, "*", "DMLC_USE_KUBERNETES", "1");
    if (rt == "worker") add_env(out, "*", "DMLC_WORKER_ID", std::to_string(index));
    return out;
  }
  if (kind == "XGBoostJob") {
    int64_t rank = index;
    if (rt == "worker") rank += spec_replicas(job, "Master");
    const std::string name = job.get("metadata").get("name").str();
    std::string master_addr = gen_general_name(name, "master", "0");
    int master_port = port_from_job(job, "Master");
    int64_t total = 0;
    for (const auto& kv : replica_specs(job).fields()) total += replicas_of(kv.second);
    add_env(out, "*", "MASTER_PORT", std::to_string(master_port));
    add_env(out, "*", "MASTER_ADDR", master_addr);
    add_env(out, "*", "WORLD_SIZE", std::to_string(total));
    add_env(out, "*", "RANK", std::to_string(rank));
    add_env(out, "*", "PYTHONUNBUFFERED", "0");
    if (total > 1) {
      int wport = port_from_job(job, "Worker");
      std::string addrs;
      for (int64_t i = 0; i < total - 1; ++i) {
        if (i) addrs += ",";
        addrs += gen_general_name(name, "worker", std::to_string(i));
      }
      add_env(out, "*", "WORKER_PORT", std::to_string(wport));
      add_env(out, "*", "WORKER_ADDRS", addrs);
    }
    return out;
  }
  return out;
}

void set_cluster_spec(const Json& job, Json& pod_template, const std::string& rtype, int index, const Options& opt) {
  Json env = gen_env(job, rtype, index, opt);
  if (env.size() == 0) return;
  Json& containers = pod_template["spec"]["containers"];
  if (!containers.is_array()) return;
  for (size_t i = 0; i < containers.size(); ++i) {
    Json& c = containers.at(i);
    const std::string cname = c.get("name").str();
    for (const auto& e : env.items()) {
      const std::string target = e.get("container").str();
      if (target != "*" && target != cname) continue;
      if (e.get("default").as_bool(false)) {  // never override the user's own setting
        bool set = false;
        const Json& cur = c.get("env");
        for (size_t j = 0; j < cur.size(); ++j) set = set || cur[j].get("name").str() == e.get("name").str();
        if (set) continue;
      }
      Json ev = Json::object();
      ev.set("name", e.get("name"));
      ev.set("value", e.get("value"));
      c["env"].push_back(ev);
    }
  }
}

}  // namespace toa
