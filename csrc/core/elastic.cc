// Elastic worker groups: spec.elasticPolicy {minReplicas, maxReplicas,
// maxRestarts, scaleUpCooldownSeconds, scaleDownDelaySeconds}.
//
// The reference only has EnableDynamicWorker (types.go:68-69; pods with index
// >= replicas are deleted and missing ones created, pod_test.go:529-685, with
// a sparse TF_CONFIG, tensorflow.go:74-83).  That works for TF's PS
// architecture, where workers join a running cluster.  An all-reduce job over
// RCCL has a FIXED world: one member disappearing hangs every collective, and
// WORLD_SIZE/RANK baked into the survivors are stale after a resize.  So the
// MI355X build treats membership changes the way torchrun's elastic agent
// does -- as GROUP restarts:
//
//   * every pod carries the label training.amd.com/elastic-generation=G and
//     the env TOA_ELASTIC_GENERATION/TOA_ELASTIC_RESTARTS;
//   * a retryable failure (exit code >= 128, or any failure under
//     OnFailure/Always), or a pod vanishing after the group launched
//     (preemption), bumps G: all pods of the old generation are deleted and,
//     once they are gone, the group is recreated with
//         replicas = clamp(min(desired, capacity), minReplicas, maxReplicas)
//     workers, so WORLD_SIZE/TF_CONFIG are rebuilt for the new size; the
//     payload resumes from TOA_CHECKPOINT_DIR (train/checkpoint.py);
//   * capacity comes from the shell (free amd.com/gpu on the nodes, counting
//     this job's own pods as free); when it grows back the group is resized
//     up after scaleUpCooldownSeconds; when it is unknown, workers stuck
//     Unschedulable for scaleDownDelaySeconds shrink the group instead;
//   * more than maxRestarts failure-driven restarts fail the job.
// Resizes do not count as restarts.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>

#include "core.h"

namespace toa {

const char* kLabelElasticGeneration = "training.amd.com/elastic-generation";

static Json act_delete_pod(const Json& p) {
  Json a = Json::object();
  a.set("op", "delete_pod");
  a.set("namespace", p.path({"metadata", "namespace"}).str("default"));
  a.set("name", p.path({"metadata", "name"}).str());
  return a;
}

static bool pod_deleting(const Json& p) { return !p.path({"metadata", "deletionTimestamp"}).is_null(); }

static int64_t pod_generation(const Json& p) {
  const std::string s = p.path({"metadata", "labels"}).get(kLabelElasticGeneration).str();
  if (s.empty()) return 0;
  return std::strtoll(s.c_str(), nullptr, 10);
}

static bool unschedulable(const Json& p) {
  if (p.path({"status", "phase"}).str() != "Pending") return false;
  for (const auto& c : p.path({"status", "conditions"}).items())
    if (c.get("type").str() == "PodScheduled" && c.get("status").str() == "False") return true;
  return false;
}

static int exit_code_of(const Json& p, const std::string& container) {
  for (const auto& cs : p.path({"status", "containerStatuses"}).items())
    if (cs.get("name").str() == container && cs.path({"state", "terminated"}).is_object())
      return (int)cs.path({"state", "terminated", "exitCode"}).as_int(1);
  return 1;
}

bool is_elastic(const Json& job) { return job.get("spec").get("elasticPolicy").is_object(); }

static void add_env(Json& tpl, const std::string& name, const std::string& value) {
  Json& spec = tpl["spec"];
  Json& cs = spec["containers"];
  for (auto& c : cs.mutable_items()) {
    Json env = c.get("env").is_array() ? c.get("env") : Json::array();
    Json e = Json::object();
    e.set("name", name);
    e.set("value", value);
    env.push_back(e);
    c.set("env", env);
  }
}

ElasticPlan elastic_prepass(Json& job, const Json& pods, Json& status, double now, const Options& opt) {
  ElasticPlan plan;
  plan.enabled = is_elastic(job);
  if (!plan.enabled) return plan;
  const KindInfo& ki = kind_info(job_kind(job));
  const Json& ep = job.get("spec").get("elasticPolicy");
  Json& specs = job["spec"][ki.specs_field];
  const std::string wt = "Worker";
  const int64_t mn = std::max<int64_t>(1, ep.get("minReplicas").as_int(1));
  const int64_t mx = std::max<int64_t>(mn, ep.get("maxReplicas").as_int(replicas_of(specs.get(wt))));
  const int64_t max_restarts = ep.get("maxRestarts").as_int(10);
  const double up_cooldown = ep.get("scaleUpCooldownSeconds").as_double(30.0);
  const double down_delay = ep.get("scaleDownDelaySeconds").as_double(30.0);
  const int64_t desired = std::min(mx, std::max(mn, replicas_of(specs.get(wt))));

  // capacity in workers (the shell passes free GPUs incl. this job's own)
  int64_t cap = mx;
  const double per_worker = pod_resource_request(specs.get(wt), opt.gpu_resource);
  if (opt.elastic_free_gpus >= 0 && per_worker > 0) {
    double other = 0;
    for (const auto& kv : specs.fields())
      if (kv.first != wt) other += pod_resource_request(kv.second, opt.gpu_resource) * (double)replicas_of(kv.second);
    cap = (int64_t)(((double)opt.elastic_free_gpus - other) / per_worker + 1e-9);
  }
  const int64_t target = std::min(mx, std::max(mn, std::min(desired, cap)));

  Json es = status.get("elasticStatus").is_object() ? status.get("elasticStatus") : Json::object();
  int64_t gen = es.get("generation").as_int(0);
  int64_t cur = es.has("currentReplicas") ? es.get("currentReplicas").as_int() : target;
  int64_t restarts = es.get("restarts").as_int(0);
  bool launched = es.get("launched").as_bool(false);
  if (!es.has("generationStartTime")) es.set("generationStartTime", rfc3339(now));

  // original restart policies decide what counts as retryable
  std::map<std::string, std::string> policy;
  for (const auto& kv : specs.fields()) policy[lower(kv.first)] = kv.second.get("restartPolicy").str();

  auto apply_size = [&](int64_t n) {
    specs[wt].set("replicas", n);
  };
  apply_size(cur);

  Json current = Json::array();
  Json stale = Json::array();
  for (const auto& p : pods.items()) (pod_generation(p) == gen ? current : stale).push_back(p);

  const bool terminal = is_succeeded(status) || is_failed(status);
  std::string reason, peer_reason;
  bool failure = false;
  if (!terminal && stale.size() == 0) {
    int64_t expected = 0;
    for (const auto& kv : specs.fields()) expected += replicas_of(kv.second);
    int64_t running = 0, succeeded = 0, present = 0;
    for (const auto& p : current.items()) {
      const std::string ph = p.path({"status", "phase"}).str();
      const std::string rt = p.path({"metadata", "labels"}).get(kLabelReplicaType).str();
      if (ph == "Running") running++;
      if (ph == "Succeeded") succeeded++;
      if (!pod_deleting(p)) present++;
      if (ph == "Failed") {
        const int code = exit_code_of(p, ki.container);
        const std::string& rp = policy[rt];
        if (is_retryable_exit_code(code) || rp == "OnFailure" || rp == "Always") {
          failure = true;
          // survivors of a lost peer exit 143 (PEER_LOST_EXIT, train/runtime.py):
          // the reason names the member whose failure started the restart
          std::string& slot = code == 143 ? peer_reason : reason;
          if (slot.empty())
            slot = p.path({"metadata", "name"}).str() + " failed with exit code " + std::to_string(code);
        }
      }
      if (launched && pod_deleting(p) && reason.empty()) {
        failure = true;
        reason = p.path({"metadata", "name"}).str() + " was preempted";
      }
    }
    if (launched && present < expected && reason.empty() && succeeded == 0) {
      failure = true;
      reason = "a member of generation " + std::to_string(gen) + " disappeared";
    }
    if (reason.empty()) reason = peer_reason;
    if (!launched && running == expected && expected > 0) {
      launched = true;
      es.set("launchTime", rfc3339(now));
      const double rs = es.get("lastRestartUnix").as_double(NAN);
      if (!std::isnan(rs)) es.set("lastResumeSeconds", now - rs);
    }
    bool resize = false;
    int64_t next = cur;
    if (!failure && succeeded == 0) {
      const double last_scale = parse_rfc3339(es.get("lastScaleTime").str(es.get("generationStartTime").str()));
      if (launched && target > cur && (std::isnan(last_scale) || now - last_scale >= up_cooldown)) {
        resize = true;
        next = target;
        reason = "scaling up to " + std::to_string(next) + " workers (capacity available)";
      } else if (!launched && target < cur) {
        resize = true;
        next = target;
        reason = "scaling down to " + std::to_string(next) + " workers (insufficient capacity)";
      } else if (!launched && cur > mn) {
        int64_t stuck = 0;
        for (const auto& p : current.items()) stuck += unschedulable(p) ? 1 : 0;
        const double gs = parse_rfc3339(es.get("generationStartTime").str());
        if (stuck > 0 && !std::isnan(gs) && now - gs >= down_delay) {
          resize = true;
          next = std::max(mn, cur - stuck);
          reason = "scaling down to " + std::to_string(next) + " workers (" + std::to_string(stuck) +
                   " unschedulable)";
        } else if (stuck > 0 && !std::isnan(gs)) {
          plan.requeue_after = std::max(0.0, gs + down_delay - now);
        }
      }
      if (launched && target > cur && std::isnan(plan.requeue_after) && !resize && !std::isnan(last_scale))
        plan.requeue_after = std::max(0.0, last_scale + up_cooldown - now);
    }
    if (failure) {
      if (restarts >= max_restarts) {
        plan.give_up = true;
        plan.message = ki.kind + " " + job.path({"metadata", "name"}).str() +
                       " has failed because it exceeded the elastic restart limit (maxRestarts=" +
                       std::to_string(max_restarts) + "): " + reason;
      } else {
        restarts++;
        next = target;
      }
    }
    if ((failure && !plan.give_up) || resize) {
      gen++;
      cur = next;
      launched = false;
      es.set("generationStartTime", rfc3339(now));
      es.erase("launchTime");
      if (failure) {
        es.set("lastRestartTime", rfc3339(now));
        es.set("lastRestartUnix", now);
      }
      else es.set("lastScaleTime", rfc3339(now));
      es.set("lastTransitionReason", reason);
      for (const auto& p : current.items()) stale.push_back(p);
      current = Json::array();
      apply_size(cur);
      plan.message = ki.kind + " " + job.path({"metadata", "name"}).str() + " is restarting as elastic generation " +
                     std::to_string(gen) + " with " + std::to_string(cur) + " workers: " + reason;
      plan.restarted = true;
    }
  }
  if (!terminal && stale.size() > 0) {
    for (const auto& p : stale.items())
      if (!pod_deleting(p)) plan.actions.push_back(act_delete_pod(p));
    plan.draining = true;
  }

  es.set("generation", gen);
  es.set("currentReplicas", cur);
  es.set("desiredReplicas", desired);
  es.set("restarts", restarts);
  es.set("launched", launched);
  if (cap != mx || opt.elastic_free_gpus >= 0) es.set("capacity", std::max<int64_t>(0, cap));
  status.set("elasticStatus", es);

  // the group's pods: generation label, env, and restartPolicy Never (the
  // operator restarts the whole group, never one member in place)
  const std::string g = std::to_string(gen);
  for (auto& kv : specs.mutable_fields()) {
    Json& tpl = kv.second["template"];
    if (!tpl.is_object()) tpl = Json::object();
    if (!tpl.get("metadata").is_object()) tpl.set("metadata", Json::object());
    if (!tpl.get("spec").is_object()) tpl.set("spec", Json::object());
    Json labels = tpl.get("metadata").get("labels").is_object() ? tpl.get("metadata").get("labels") : Json::object();
    labels.set(kLabelElasticGeneration, g);
    tpl["metadata"].set("labels", labels);
    add_env(tpl, "TOA_ELASTIC_GENERATION", g);
    add_env(tpl, "TOA_ELASTIC_RESTARTS", std::to_string(restarts));
    kv.second.set("restartPolicy", "Never");
  }
  plan.pods = terminal ? pods : current;
  return plan;
}

}  // namespace toa
