// Job status engines (one per kind), run after ReconcilePods has refreshed
// status.replicaStatuses.  Truth table oracle: SURVEY Appendix A
// (pkg/controller.v1/tensorflow/status_test.go:120-425).
//
// Deliberate fixes vs the reference: one TF engine instead of
// two copies (quirk 9); MX/XGB/PyTorch write completionTime into the status
// they return (quirk 6); metrics count condition TRANSITIONS, not syncs.
#include "core.h"

namespace toa {

static int64_t rs_get(const Json& status, const std::string& rt, const char* f) {
  return status.path({"replicaStatuses"}).get(rt).get(f).as_int(0);
}

static void set_completion(Json& status, double now) {
  if (status.get("completionTime").is_null()) status.set("completionTime", rfc3339(now));
}

static void event(StatusResult& out, const std::string& type, const std::string& reason, const std::string& msg) {
  Json e = Json::object();
  e.set("type", type);
  e.set("reason", reason);
  e.set("message", msg);
  out.events.push_back(e);
}

// worker-0 exited 0 and its pod Succeeded (tensorflow/pod.go:361-381)
static bool worker0_completed(const Json& job, const Json& pods) {
  const KindInfo& ki = kind_info(job_kind(job));
  if (!replica_specs(job).has("Worker")) return true;
  for (const auto& p : pods.items()) {
    const Json& lb = p.path({"metadata", "labels"});
    if (lb.get(kLabelReplicaType).str() != "worker" || lb.get(kLabelReplicaIndex).str() != "0") continue;
    int64_t code = 0xbeef;
    for (const auto& cs : p.path({"status", "containerStatuses"}).items())
      if (cs.get("name").str() == ki.container && cs.path({"state", "terminated"}).is_object())
        code = cs.path({"state", "terminated", "exitCode"}).as_int(0xbeef);
    if (code == 0 && p.path({"status", "phase"}).str() == "Succeeded") return true;
  }
  return false;
}

static void tf_status(const Json& job, const Json& pods, Json& status, double now, StatusResult& out) {
  const Json& md = job.get("metadata");
  const std::string jn = md.get("namespace").str("default") + "/" + md.get("name").str();
  const Json& specs = replica_specs(job);
  const bool w0 = worker0_completed(job, pods);
  const bool has_chief = specs.has("Chief") || specs.has("Master");
  const bool all_workers = job.get("spec").get("successPolicy").str() == "AllWorkers";
  for (const char* rtc : {"Chief", "Evaluator", "Master", "PS", "Worker"}) {
    const std::string rt = rtc;
    const Json* sp = specs.find(rt);
    if (!sp || sp->is_null()) continue;
    const int64_t succeeded = rs_get(status, rt, "succeeded");
    const int64_t expected = replicas_of(*sp) - succeeded;
    const int64_t running = rs_get(status, rt, "active");
    const int64_t failed = rs_get(status, rt, "failed");
    if (has_chief) {
      if (is_chief_or_master(rt)) {
        if (running > 0) update_job_conditions(status, "Running", "TFJobRunning", "TFJob " + jn + " is running.", now);
        if (expected == 0) {
          std::string msg = "TFJob " + jn + " successfully completed.";
          set_completion(status, now);
          if (update_job_conditions(status, "Succeeded", "TFJobSucceeded", msg, now)) {
            event(out, "Normal", "TFJobSucceeded", msg);
            out.succeeded++;
          }
        }
      }
    } else if (rt == "Worker") {
      if (expected == 0 || (w0 && !all_workers)) {
        std::string msg = "TFJob " + jn + " successfully completed.";
        set_completion(status, now);
        if (update_job_conditions(status, "Succeeded", "TFJobSucceeded", msg, now)) {
          event(out, "Normal", "TFJobSucceeded", msg);
          out.succeeded++;
        }
      } else if (running > 0) {
        update_job_conditions(status, "Running", "TFJobRunning", "TFJob " + jn + " is running.", now);
      }
    }
    if (failed > 0) {
      if (!has_condition(status, "Restarting")) {
        std::string msg = "TFJob " + jn + " has failed because " + std::to_string(failed) + " " + rt +
                          " replica(s) failed.";
        set_completion(status, now);
        if (update_job_conditions(status, "Failed", "TFJobFailed", msg, now)) {
          event(out, "Normal", "TFJobFailed", msg);
          out.failed++;
        }
      }
    }
  }
}

// PyTorchJob / XGBoostJob: Master drives Running/Succeeded; then "Running" always.
static void master_worker_status(const Json& job, Json& status, double now, StatusResult& out) {
  const std::string kind = job_kind(job);
  const bool pt = kind == "PyTorchJob";
  const std::string name = job.path({"metadata", "name"}).str();
  const std::string pre = pt ? "Job" : "XGBoostJob";
  const std::string noun = pt ? "PyTorchJob " : "XGBoostJob ";
  const Json& specs = replica_specs(job);
  for (const char* rtc : {"Master", "Worker"}) {
    const std::string rt = rtc;
    const Json* sp = specs.find(rt);
    if (!sp || sp->is_null()) continue;
    const int64_t succeeded = rs_get(status, rt, "succeeded");
    const int64_t expected = replicas_of(*sp) - succeeded;
    const int64_t running = rs_get(status, rt, "active");
    const int64_t failed = rs_get(status, rt, "failed");
    if (rt == "Master") {
      if (running > 0) update_job_conditions(status, "Running", pre + "Running", noun + name + " is running.", now);
      if (expected == 0) {
        std::string msg = noun + name + " is successfully completed.";
        set_completion(status, now);
        if (update_job_conditions(status, "Succeeded", pre + "Succeeded", msg, now)) {
          event(out, "Normal", pre + "Succeeded", msg);
          out.succeeded++;
        }
        return;
      }
    }
    if (failed > 0) {
      if (sp->get("restartPolicy").str() == "ExitCode") {
        std::string msg = noun + name + " is restarting because " + std::to_string(failed) + " " + rt +
                          " replica(s) failed.";
        if (update_job_conditions(status, "Restarting", pre + "Restarting", msg, now))
          event(out, "Warning", pre + "Restarting", msg);
      } else {
        std::string msg = noun + name + " is failed because " + std::to_string(failed) + " " + rt +
                          " replica(s) failed.";
        set_completion(status, now);
        if (update_job_conditions(status, "Failed", pre + "Failed", msg, now)) {
          event(out, "Normal", pre + "Failed", msg);
          out.failed++;
        }
      }
    }
  }
  update_job_conditions(status, "Running", pre + "Running", noun + name + " is running.", now);
}

// MXJob: every replica type can drive Running / Succeeded (mxjob_controller.go:328-410)
static void mx_status(const Json& job, Json& status, double now, StatusResult& out) {
  const std::string name = job.path({"metadata", "name"}).str();
  const Json& specs = replica_specs(job);
  for (const auto& rtc : kind_info("MXJob").replica_types) {
    const std::string rt = rtc;
    const Json* sp = specs.find(rt);
    if (!sp || sp->is_null()) continue;
    const int64_t succeeded = rs_get(status, rt, "succeeded");
    const int64_t expected = replicas_of(*sp) - succeeded;
    const int64_t running = rs_get(status, rt, "active");
    const int64_t failed = rs_get(status, rt, "failed");
    if (running > 0) update_job_conditions(status, "Running", "MXJobRunning", "MXJob " + name + " is running.", now);
    if (expected == 0) {
      std::string msg = "MXJob " + name + " is successfully completed.";
      set_completion(status, now);
      if (update_job_conditions(status, "Succeeded", "MXJobSucceeded", msg, now)) {
        event(out, "Normal", "MXJobSucceeded", msg);
        out.succeeded++;
      }
    }
    if (failed > 0) {
      if (sp->get("restartPolicy").str() == "ExitCode") {
        std::string msg = "mxjob " + name + " is restarting because " + std::to_string(failed) + " " + rt +
                          " replica(s) failed.";
        if (update_job_conditions(status, "Restarting", "MXJobRestarting", msg, now))
          event(out, "Warning", "MXJobRestarting", msg);
      } else {
        std::string msg = "mxjob " + name + " is failed because " + std::to_string(failed) + " " + rt +
                          " replica(s) failed.";
        set_completion(status, now);
        if (update_job_conditions(status, "Failed", "MXJobFailed", msg, now)) {
          event(out, "Normal", "MXJobFailed", msg);
          out.failed++;
        }
      }
    }
  }
}

void update_job_status(const Json& job, const Json& pods, Json& status, double now, StatusResult& out) {
  const std::string kind = job_kind(job);
  if (status.get("startTime").is_null()) status.set("startTime", rfc3339(now));
  if (kind == "TFJob") tf_status(job, pods, status, now, out);
  else if (kind == "MXJob") mx_status(job, status, now, out);
  else master_worker_status(job, status, now, out);
}

}  // namespace toa
