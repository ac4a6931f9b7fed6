// Native informer cache + rate-limited work queue.
//
// Store:      indexed object cache keyed "ns/name" with a namespace index and
//             label-selector listing (the lister/indexer half of a client-go
//             informer; reference pkg/client/listers/tensorflow/v1/tfjob.go:43-97).
// WorkQueue:  de-duplicating, delayed, per-item exponential-backoff queue
//             (client-go workqueue.RateLimitingInterface used by the legacy
//             controller, pkg/controller.v1/tensorflow/controller.go:193-286;
//             the new binary's FakeWorkQueue no-op is replaced by this).
#pragma once
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "json.h"

namespace toa {

class Store {
 public:
  // returns true if the object is new or its resourceVersion changed
  bool upsert(const Json& obj);
  bool remove(const std::string& key);
  bool get(const std::string& key, Json* out) const;
  std::vector<Json> list(const std::string& ns, const Json& selector) const;  // selector: {k: v}
  std::vector<std::string> keys() const;
  size_t size() const;
  static std::string key_of(const Json& obj);

 private:
  mutable std::mutex mu_;
  std::map<std::string, Json> items_;
  std::map<std::string, std::set<std::string>> by_ns_;
};

class WorkQueue {
 public:
  WorkQueue(double base_delay = 0.005, double max_delay = 1000.0) : base_(base_delay), max_(max_delay) {}
  void add(const std::string& key);
  void add_after(const std::string& key, double delay_s);
  void add_rate_limited(const std::string& key);
  void forget(const std::string& key);
  int num_requeues(const std::string& key) const;
  // blocks up to timeout_s; returns false on timeout or shutdown
  bool get(std::string* key, double timeout_s);
  void done(const std::string& key);
  size_t len() const;
  void shutdown();
  bool shutting_down() const;

 private:
  void promote_locked(double now);
  double now_s() const;
  double base_, max_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::string> queue_;
  std::set<std::string> dirty_, processing_;
  std::multimap<double, std::string> delayed_;
  std::map<std::string, int> failures_;
  bool shutdown_ = false;
};

}  // namespace toa
