// Job conditions + RFC3339 time helpers.
//
// Semantics of UpdateJobConditions ([EXT] kubeflow/common util/status.go,
// pinned by pkg/controller.v1/tensorflow/status_test.go:585-592 and the SDK
// reading conditions[-1], sdk/python/kubeflow/tfjob/api/tf_job_client.py:317):
//   * a Failed (and here also a Succeeded) job is frozen,
//   * no-op when the same type already has the same status and reason,
//   * the old condition of that type is removed, Running <-> Restarting are
//     mutually exclusive, Running flips to False when Succeeded/Failed lands,
//   * the new condition is appended LAST; lastTransitionTime is kept when the
//     status of that type did not change.
#include <cmath>
#include <cstdio>
#include <ctime>

#include "core.h"

namespace toa {

std::string rfc3339(double t) {
  time_t s = (time_t)std::floor(t);
  struct tm tmv;
  gmtime_r(&s, &tmv);
  char buf[32];
  strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%SZ", &tmv);
  return buf;
}

double parse_rfc3339(const std::string& s) {
  int Y, M, D, h, m;
  double sec;
  char tz[16] = {0};
  if (sscanf(s.c_str(), "%d-%d-%dT%d:%d:%lf%15s", &Y, &M, &D, &h, &m, &sec, tz) < 6) return NAN;
  struct tm tmv = {};
  tmv.tm_year = Y - 1900;
  tmv.tm_mon = M - 1;
  tmv.tm_mday = D;
  tmv.tm_hour = h;
  tmv.tm_min = m;
  tmv.tm_sec = 0;
  double t = (double)timegm(&tmv) + sec;
  // numeric offsets (+hh:mm / -hh:mm); 'Z' or empty = UTC
  if (tz[0] == '+' || tz[0] == '-') {
    int oh = 0, om = 0;
    sscanf(tz + 1, "%d:%d", &oh, &om);
    double off = oh * 3600.0 + om * 60.0;
    t += (tz[0] == '+') ? -off : off;
  }
  return t;
}

static const Json* find_condition(const Json& status, const std::string& type) {
  for (const auto& c : status.get("conditions").items())
    if (c.get("type").str() == type) return &c;
  return nullptr;
}

bool has_condition(const Json& status, const std::string& type) {
  for (const auto& c : status.get("conditions").items())
    if (c.get("type").str() == type && c.get("status").str() == "True") return true;
  return false;
}

bool is_succeeded(const Json& status) { return has_condition(status, "Succeeded"); }
bool is_failed(const Json& status) { return has_condition(status, "Failed"); }

bool update_job_conditions(Json& status, const std::string& type, const std::string& reason, const std::string& msg,
                           double now) {
  // Terminal conditions are sticky.  The reference only freezes Failed jobs;
  // freezing Succeeded too keeps e.g. "chief succeeded, workers then killed"
  // a Succeeded job (status_test.go:402-425 expects Succeeded there, which the
  // reference only satisfies because it checks presence, not the last entry).
  if (is_failed(status) || is_succeeded(status)) return false;
  const std::string ts = rfc3339(now);
  Json cond = Json::object();
  cond.set("type", type);
  cond.set("status", "True");
  cond.set("reason", reason);
  cond.set("message", msg);
  cond.set("lastUpdateTime", ts);
  cond.set("lastTransitionTime", ts);
  const Json* cur = find_condition(status, type);
  if (cur && cur->get("status").str() == "True" && cur->get("reason").str() == reason) return false;
  if (cur && cur->get("status").str() == "True") cond.set("lastTransitionTime", cur->get("lastTransitionTime"));
  Json out = Json::array();
  for (const auto& c0 : status.get("conditions").items()) {
    const std::string ct = c0.get("type").str();
    if (type == "Restarting" && ct == "Running") continue;
    if (type == "Running" && ct == "Restarting") continue;
    if (ct == type) continue;
    Json c = c0;
    if ((type == "Failed" || type == "Succeeded") && ct == "Running" && c.get("status").str() == "True") {
      c.set("status", "False");
      c.set("lastTransitionTime", ts);
    }
    out.push_back(c);
  }
  out.push_back(cond);
  status.set("conditions", out);
  return true;
}

}  // namespace toa
