// Controller expectations (client-go ControllerExpectations semantics):
// per key, the number of creations / deletions the controller issued but has
// not yet observed through the watch.  A key is "satisfied" when both counts
// reached <= 0, when it does not exist, or when the record is older than the
// TTL (5 min -- lost watch events must not wedge a job forever).
//
// Keys: "<ns>/<job>/<rt-lower>/pods" and ".../services" (pinned by
// pkg/controller.v1/tensorflow/pod_test.go:151-165).  Unlike the reference
// glue (pkg/common/util/reconciler.go:23-35) the shell checks
// ALL replica types with AND semantics and the same lower-case keys the
// creator used.
#include "core.h"

namespace toa {

std::string expectation_pods_key(const std::string& job_key, const std::string& rt_lower) {
  return job_key + "/" + rt_lower + "/pods";
}
std::string expectation_services_key(const std::string& job_key, const std::string& rt_lower) {
  return job_key + "/" + rt_lower + "/services";
}

void Expectations::expect_creations(const std::string& key, int n, double now) {
  std::lock_guard<std::mutex> g(mu_);
  auto& r = m_[key];
  // client-go SetExpectations overwrites; ExpectCreations raises from the
  // current record when it is still pending.
  if (r.add <= 0 && r.del <= 0) {
    r.add = 0;
    r.del = 0;
  }
  r.add += n;
  r.ts = now;
}

void Expectations::expect_deletions(const std::string& key, int n, double now) {
  std::lock_guard<std::mutex> g(mu_);
  auto& r = m_[key];
  if (r.add <= 0 && r.del <= 0) {
    r.add = 0;
    r.del = 0;
  }
  r.del += n;
  r.ts = now;
}

void Expectations::creation_observed(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = m_.find(key);
  if (it != m_.end()) it->second.add--;
}

void Expectations::deletion_observed(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = m_.find(key);
  if (it != m_.end()) it->second.del--;
}

bool Expectations::satisfied(const std::string& key, double now) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = m_.find(key);
  if (it == m_.end()) return true;
  const Rec& r = it->second;
  if (r.add <= 0 && r.del <= 0) return true;
  return now - r.ts > ttl_;
}

void Expectations::delete_key(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  m_.erase(key);
}

std::pair<int64_t, int64_t> Expectations::get(const std::string& key) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = m_.find(key);
  if (it == m_.end()) return {0, 0};
  return {it->second.add, it->second.del};
}

bool Expectations::exists(const std::string& key) const {
  std::lock_guard<std::mutex> g(mu_);
  return m_.count(key) > 0;
}

}  // namespace toa
