// Native self-test of the operator core, built with sanitizers
// (ASan+UBSan, and TSan for the concurrent WorkQueue / Store / Expectations):
//   g++ -std=c++17 -fsanitize=address,undefined ...   (tests/test_core_sanitizers.py)
// It drives reconcile() over a randomized grid of pod phase / exit-code /
// restart-count combinations for every kind (a property test: the engine
// must never crash, must never emit duplicate creates, and a terminal job
// must never get Running back), then hammers the queue from several threads.
#include <atomic>
#include <cstdlib>
#include <cstdio>
#include <random>
#include <set>
#include <thread>

#include "../core.h"
#include "../store.h"

using namespace toa;

static int failures = 0;
#define CHECK(c)                                                              \
  do {                                                                        \
    if (!(c)) {                                                               \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);    \
      ++failures;                                                             \
    }                                                                         \
  } while (0)

static Json make_job(const std::string& kind, std::mt19937& rng) {
  const KindInfo& ki = kind_info(kind);
  Json job = Json::object();
  job.set("apiVersion", "kubeflow.org/v1");
  job.set("kind", kind);
  Json md = Json::object();
  md.set("name", "job-" + std::to_string(rng() % 1000));
  md.set("namespace", "ns");
  md.set("uid", "uid-1");
  job.set("metadata", md);
  Json specs = Json::object();
  std::vector<std::string> types = ki.replica_types;
  for (const auto& t : types) {
    if (kind == "TFJob" && (t == "Master" || t == "Evaluator") && rng() % 2) continue;
    if (kind == "MXJob" && t.rfind("Tuner", 0) == 0) continue;
    if (rng() % 3 == 0 && t != "Master" && t != "Worker") continue;
    Json rs = Json::object();
    int64_t n = (t == "Master" || t == "Chief" || t == "Scheduler") ? 1 : 1 + rng() % 4;
    rs.set("replicas", n);
    const char* rps[] = {"Never", "OnFailure", "Always", "ExitCode"};
    rs.set("restartPolicy", rps[rng() % 4]);
    Json c = Json::object();
    c.set("name", ki.container);
    c.set("image", "img");
    Json cs = Json::array();
    cs.push_back(c);
    Json ps = Json::object();
    ps.set("containers", cs);
    Json tpl = Json::object();
    tpl.set("spec", ps);
    rs.set("template", tpl);
    specs.set(t, rs);
  }
  Json spec = Json::object();
  spec.set(ki.specs_field, specs);
  Json rp = Json::object();
  if (rng() % 3 == 0) rp.set("backoffLimit", (int64_t)(rng() % 4));
  if (rng() % 3 == 0) rp.set("activeDeadlineSeconds", (int64_t)(rng() % 100));
  if (rng() % 3 == 0) rp.set("ttlSecondsAfterFinished", (int64_t)(rng() % 100));
  spec.set("runPolicy", rp);
  job.set("spec", spec);
  return job;
}

static Json make_pods(const Json& job, std::mt19937& rng) {
  Json pods = Json::array();
  const KindInfo& ki = kind_info(job_kind(job));
  for (const auto& kv : replica_specs(job).fields()) {
    int64_t n = replicas_of(kv.second) + (int64_t)(rng() % 2);
    for (int64_t i = 0; i < n; ++i) {
      if (rng() % 4 == 0) continue;
      Json p = Json::object();
      Json md = Json::object();
      md.set("name", lower(kv.first) + "-" + std::to_string(i));
      md.set("namespace", "ns");
      Json lb = Json::object();
      lb.set(kLabelReplicaType, lower(kv.first));
      lb.set(kLabelReplicaIndex, std::to_string(i));
      md.set("labels", lb);
      p.set("metadata", md);
      const char* phases[] = {"Pending", "Running", "Succeeded", "Failed", "Unknown"};
      Json st = Json::object();
      st.set("phase", phases[rng() % 5]);
      Json css = Json::array();
      Json cst = Json::object();
      cst.set("name", ki.container);
      cst.set("restartCount", (int64_t)(rng() % 3));
      if (rng() % 2) {
        Json term = Json::object();
        const int codes[] = {0, 1, 2, 127, 128, 130, 137, 143};
        term.set("exitCode", (int64_t)codes[rng() % 8]);
        Json state = Json::object();
        state.set("terminated", term);
        cst.set("state", state);
      }
      css.push_back(cst);
      st.set("containerStatuses", css);
      p.set("status", st);
      pods.push_back(p);
    }
  }
  return pods;
}

static void property_reconcile() {
  std::mt19937 rng(1234);
  Options opt;
  const int iters = getenv("TOA_SELFTEST_ITERS") ? atoi(getenv("TOA_SELFTEST_ITERS")) : 3000;
  for (int it = 0; it < iters; ++it) {
    for (const auto& kind : supported_kinds()) {
      Json job = on_job_created(make_job(kind, rng), 1000.0);
      opt.enable_gang_scheduling = rng() % 2;
      opt.previous_retry = (int)(rng() % 3);
      Json status = job.get("status");
      for (int pass = 0; pass < 3; ++pass) {
        Json pods = make_pods(job, rng);
        Json res = reconcile(job, pods, Json::array(), 1000.0 + pass * 40.0, opt);
        std::set<std::string> created;
        for (const auto& a : res.get("actions").items()) {
          if (a.get("op").str() != "create_pod") continue;
          const std::string n = a.path({"pod", "metadata", "name"}).str();
          CHECK(!created.count(n));
          created.insert(n);
        }
        const Json& ns = res.get("status");
        const bool was_terminal = is_succeeded(status) || is_failed(status);
        if (was_terminal) {
          CHECK(is_succeeded(ns) || is_failed(ns));
          for (const auto& c : ns.get("conditions").items())
            if (c.get("type").str() == "Running") CHECK(c.get("status").str() != "True");
        }
        // at most one of Succeeded/Failed is True
        CHECK(!(is_succeeded(ns) && is_failed(ns)));
        job.set("status", ns);
        status = ns;
        // round trip through text must be lossless
        CHECK(Json::parse(res.dump()) == res);
      }
    }
  }
}

static void concurrency() {
  WorkQueue q(0.0001, 0.01);
  Store store;
  Expectations exp;
  std::atomic<int> processed{0};
  std::vector<std::thread> ts;
  for (int w = 0; w < 4; ++w) {
    ts.emplace_back([&, w] {
      std::string k;
      while (q.get(&k, 0.2)) {
        Json o = Json::object();
        Json md = Json::object();
        md.set("name", k);
        md.set("namespace", "ns");
        md.set("resourceVersion", std::to_string(w));
        o.set("metadata", md);
        store.upsert(o);
        exp.creation_observed("ns/" + k + "/worker/pods");
        processed++;
        if (processed % 7 == 0) q.add_rate_limited(k);
        else q.forget(k);
        q.done(k);
      }
    });
  }
  for (int p = 0; p < 2; ++p) {
    ts.emplace_back([&, p] {
      for (int i = 0; i < 2000; ++i) {
        std::string k = "job-" + std::to_string((i * 7 + p) % 97);
        exp.expect_creations("ns/" + k + "/worker/pods", 1, 0.0);
        if (i % 3) q.add(k);
        else q.add_after(k, 0.001);
        (void)store.list("ns", Json::object());
      }
    });
  }
  for (size_t i = 4; i < ts.size(); ++i) ts[i].join();
  std::this_thread::sleep_for(std::chrono::milliseconds(300));
  q.shutdown();
  for (int i = 0; i < 4; ++i) ts[i].join();
  CHECK(processed > 0);
  CHECK(store.size() <= 97);
}

int main() {
  property_reconcile();
  concurrency();
  // JSON edge cases
  CHECK(Json::parse("{\"a\":\"<&>\"}").dump() == "{\"a\":\"\\u003c\\u0026\\u003e\"}");
  CHECK(Json::parse("[1,2.5,-3,true,null,\"\\u00e9\"]").dump() == "[1,2.5,-3,true,null,\"\xc3\xa9\"]");
  bool threw = false;
  try {
    Json::parse("{\"a\":");
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw);
  if (failures) {
    fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  printf("core selftest OK\n");
  return 0;
}
