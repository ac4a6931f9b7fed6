// pybind11 bindings of the operator core (module tf_operator_amd.core._toa_core).
// Objects cross the boundary as JSON text; tf_operator_amd/core/__init__.py
// wraps these with dict-in / dict-out helpers.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "core.h"
#include "store.h"

namespace py = pybind11;
using namespace toa;

static Json J(const std::string& s) { return s.empty() ? Json() : Json::parse(s); }

PYBIND11_MODULE(_toa_core, m) {
  m.doc() = "tf_operator_amd C++17 operator core (pure, I/O-free reconcile engine)";
  m.attr("API_VERSION") = kApiVersion;
  m.attr("GROUP") = kGroup;
  m.attr("VERSION") = kVersion;

  m.def("supported_kinds", &supported_kinds);
  m.def("kind_info", [](const std::string& k) {
    const KindInfo& ki = kind_info(k);
    py::dict d;
    d["kind"] = ki.kind;
    d["plural"] = ki.plural;
    d["singular"] = ki.singular;
    d["specs_field"] = ki.specs_field;
    d["container"] = ki.container;
    d["port_name"] = ki.port_name;
    d["port"] = ki.port;
    d["default_restart"] = ki.default_restart;
    d["default_clean"] = ki.default_clean;
    d["replica_types"] = ki.replica_types;
    d["reason_prefix"] = ki.reason_prefix;
    d["controller_name"] = ki.controller_name;
    return d;
  });
  m.def("set_defaults", [](const std::string& job) { return set_defaults(J(job)).dump(); });
  m.def("validate", [](const std::string& job) { return validate(J(job)); });
  m.def("on_job_created", [](const std::string& job, double now) { return on_job_created(J(job), now).dump(); });
  m.def("claim_objects", [](const std::string& job, const std::string& objs) {
    return claim_objects(set_defaults(J(job)), J(objs)).dump();
  });
  m.def(
      "reconcile",
      [](const std::string& job, const std::string& pods, const std::string& services, double now,
         const std::string& options) {
        Json j = J(job), p = J(pods), s = J(services), o = J(options);
        std::string out;
        {
          py::gil_scoped_release nogil;
          out = reconcile(j, p.is_null() ? Json::array() : p, s.is_null() ? Json::array() : s, now,
                          options_from_json(o))
                    .dump();
        }
        return out;
      },
      py::arg("job"), py::arg("pods"), py::arg("services"), py::arg("now"), py::arg("options") = "");
  m.def(
      "gen_tf_config",
      [](const std::string& job, const std::string& rt, int index, const std::string& options) {
        Json j = set_defaults(J(job));
        return gen_tf_config(j, lower(rt), index, options_from_json(J(options)));
      },
      py::arg("job"), py::arg("rtype"), py::arg("index"), py::arg("options") = "");
  m.def(
      "gen_env",
      [](const std::string& job, const std::string& rtype, int index, const std::string& options) {
        Json j = set_defaults(J(job));
        return gen_env(j, rtype, index, options_from_json(J(options))).dump();
      },
      py::arg("job"), py::arg("rtype"), py::arg("index"), py::arg("options") = "");
  m.def(
      "set_cluster_spec",
      [](const std::string& job, const std::string& tpl, const std::string& rtype, int index,
         const std::string& options) {
        Json t = J(tpl);
        set_cluster_spec(set_defaults(J(job)), t, rtype, index, options_from_json(J(options)));
        return t.dump();
      },
      py::arg("job"), py::arg("template"), py::arg("rtype"), py::arg("index"), py::arg("options") = "");
  m.def(
      "node_local",
      [](const std::string& job, const std::string& options) {
        return node_local(set_defaults(J(job)), options_from_json(J(options)));
      },
      py::arg("job"), py::arg("options") = "{}");
  m.def("tf_is_distributed", [](const std::string& job) { return tf_is_distributed(set_defaults(J(job))); });
  m.def(
      "gen_podgroup",
      [](const std::string& job, const std::string& options) {
        return gen_podgroup(set_defaults(J(job)), options_from_json(J(options))).dump();
      },
      py::arg("job"), py::arg("options") = "");
  m.def("update_job_conditions",
        [](const std::string& status, const std::string& type, const std::string& reason, const std::string& msg,
           double now) {
          Json st = J(status);
          if (st.is_null()) st = Json::object();
          bool ch = update_job_conditions(st, type, reason, msg, now);
          return py::make_tuple(st.dump(), ch);
        });
  m.def("is_retryable_exit_code", &is_retryable_exit_code);
  m.def("rfc3339", &rfc3339);
  m.def("parse_rfc3339", &parse_rfc3339);
  m.def("gen_general_name", &gen_general_name);
  m.def("expectation_pods_key", &expectation_pods_key);
  m.def("expectation_services_key", &expectation_services_key);
  m.def("json_roundtrip", [](const std::string& s, bool sort) { return Json::parse(s).dump(sort); });

  py::class_<Expectations>(m, "Expectations")
      .def(py::init<double>(), py::arg("ttl_seconds") = 300.0)
      .def("expect_creations", &Expectations::expect_creations)
      .def("expect_deletions", &Expectations::expect_deletions)
      .def("creation_observed", &Expectations::creation_observed)
      .def("deletion_observed", &Expectations::deletion_observed)
      .def("satisfied", &Expectations::satisfied)
      .def("delete_key", &Expectations::delete_key)
      .def("get", &Expectations::get)
      .def("exists", &Expectations::exists);

  py::class_<Store>(m, "Store")
      .def(py::init<>())
      .def("upsert", [](Store& s, const std::string& obj) { return s.upsert(J(obj)); })
      .def("remove", &Store::remove)
      .def("get",
           [](const Store& s, const std::string& key) -> py::object {
             Json out;
             if (!s.get(key, &out)) return py::none();
             return py::str(out.dump());
           })
      .def(
          "list",
          [](const Store& s, const std::string& ns, const std::string& selector) {
            Json sel = J(selector);
            Json arr = Json::array();
            for (auto& o : s.list(ns, sel.is_null() ? Json::object() : sel)) arr.push_back(o);
            return arr.dump();
          },
          py::arg("namespace") = "", py::arg("selector") = "")
      .def("keys", &Store::keys)
      .def("__len__", &Store::size)
      .def_static("key_of", [](const std::string& obj) { return Store::key_of(J(obj)); });

  py::class_<WorkQueue>(m, "WorkQueue")
      .def(py::init<double, double>(), py::arg("base_delay") = 0.005, py::arg("max_delay") = 1000.0)
      .def("add", &WorkQueue::add)
      .def("add_after", &WorkQueue::add_after)
      .def("add_rate_limited", &WorkQueue::add_rate_limited)
      .def("forget", &WorkQueue::forget)
      .def("num_requeues", &WorkQueue::num_requeues)
      .def(
          "get",
          [](WorkQueue& q, double timeout) -> py::object {
            std::string k;
            bool ok;
            {
              py::gil_scoped_release nogil;
              ok = q.get(&k, timeout);
            }
            if (!ok) return py::none();
            return py::str(k);
          },
          py::arg("timeout") = 1.0)
      .def("done", &WorkQueue::done)
      .def("__len__", &WorkQueue::len)
      .def("shutdown", &WorkQueue::shutdown)
      .def("shutting_down", &WorkQueue::shutting_down);
}
