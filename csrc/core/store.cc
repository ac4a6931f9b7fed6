#include "store.h"

#include <chrono>
#include <cmath>

namespace toa {

std::string Store::key_of(const Json& obj) {
  const Json& md = obj.get("metadata");
  std::string ns = md.get("namespace").str();
  std::string name = md.get("name").str();
  return ns.empty() ? name : ns + "/" + name;
}

bool Store::upsert(const Json& obj) {
  std::lock_guard<std::mutex> g(mu_);
  const std::string k = key_of(obj);
  auto it = items_.find(k);
  bool changed = true;
  if (it != items_.end()) {
    const std::string rv_old = it->second.path({"metadata", "resourceVersion"}).str();
    const std::string rv_new = obj.path({"metadata", "resourceVersion"}).str();
    changed = rv_old.empty() || rv_old != rv_new;
  }
  items_[k] = obj;
  by_ns_[obj.path({"metadata", "namespace"}).str()].insert(k);
  return changed;
}

bool Store::remove(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = items_.find(key);
  if (it == items_.end()) return false;
  by_ns_[it->second.path({"metadata", "namespace"}).str()].erase(key);
  items_.erase(it);
  return true;
}

bool Store::get(const std::string& key, Json* out) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = items_.find(key);
  if (it == items_.end()) return false;
  *out = it->second;
  return true;
}

static bool matches(const Json& obj, const Json& sel) {
  const Json& labels = obj.path({"metadata", "labels"});
  for (const auto& kv : sel.fields())
    if (labels.get(kv.first).str() != kv.second.str()) return false;
  return true;
}

std::vector<Json> Store::list(const std::string& ns, const Json& selector) const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<Json> out;
  if (ns.empty()) {
    for (const auto& kv : items_)
      if (matches(kv.second, selector)) out.push_back(kv.second);
    return out;
  }
  auto it = by_ns_.find(ns);
  if (it == by_ns_.end()) return out;
  for (const auto& k : it->second) {
    const Json& o = items_.at(k);
    if (matches(o, selector)) out.push_back(o);
  }
  return out;
}

std::vector<std::string> Store::keys() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  for (const auto& kv : items_) out.push_back(kv.first);
  return out;
}

size_t Store::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return items_.size();
}

// ---------------------------------------------------------------------------
double WorkQueue::now_s() const {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

void WorkQueue::add(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  if (shutdown_) return;
  if (dirty_.count(key)) return;
  dirty_.insert(key);
  if (processing_.count(key)) return;  // re-queued when done()
  queue_.push_back(key);
  cv_.notify_one();
}

void WorkQueue::add_after(const std::string& key, double delay_s) {
  if (delay_s <= 0) {
    add(key);
    return;
  }
  std::lock_guard<std::mutex> g(mu_);
  if (shutdown_) return;
  delayed_.emplace(now_s() + delay_s, key);
  cv_.notify_one();
}

void WorkQueue::add_rate_limited(const std::string& key) {
  double d;
  {
    std::lock_guard<std::mutex> g(mu_);
    int f = failures_[key]++;
    d = base_ * std::pow(2.0, f);
    if (d > max_) d = max_;
  }
  add_after(key, d);
}

void WorkQueue::forget(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  failures_.erase(key);
}

int WorkQueue::num_requeues(const std::string& key) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = failures_.find(key);
  return it == failures_.end() ? 0 : it->second;
}

void WorkQueue::promote_locked(double now) {
  while (!delayed_.empty() && delayed_.begin()->first <= now) {
    std::string k = delayed_.begin()->second;
    delayed_.erase(delayed_.begin());
    if (dirty_.count(k)) continue;
    dirty_.insert(k);
    if (!processing_.count(k)) queue_.push_back(k);
  }
}

bool WorkQueue::get(std::string* key, double timeout_s) {
  std::unique_lock<std::mutex> lk(mu_);
  const double deadline = now_s() + timeout_s;
  while (true) {
    promote_locked(now_s());
    if (!queue_.empty()) break;
    if (shutdown_) return false;
    double now = now_s();
    if (now >= deadline) return false;
    double wait = deadline - now;
    if (!delayed_.empty()) wait = std::min(wait, std::max(0.0, delayed_.begin()->first - now));
    // system_clock deadline -> pthread_cond_timedwait (steady-clock waits use
    // pthread_cond_clockwait, which GCC 11's TSan runtime does not intercept)
    cv_.wait_until(lk, std::chrono::system_clock::now() +
                           std::chrono::duration_cast<std::chrono::system_clock::duration>(
                               std::chrono::duration<double>(wait)));
  }
  *key = queue_.front();
  queue_.pop_front();
  processing_.insert(*key);
  dirty_.erase(*key);
  return true;
}

void WorkQueue::done(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  processing_.erase(key);
  if (dirty_.count(key)) {
    queue_.push_back(key);
    cv_.notify_one();
  }
}

size_t WorkQueue::len() const {
  std::lock_guard<std::mutex> g(mu_);
  return queue_.size();
}

void WorkQueue::shutdown() {
  std::lock_guard<std::mutex> g(mu_);
  shutdown_ = true;
  cv_.notify_all();
}

bool WorkQueue::shutting_down() const {
  std::lock_guard<std::mutex> g(mu_);
  return shutdown_;
}

}  // namespace toa
