// ControllerRef claiming: which pods / services a job owns.
//
// Re-implements client-go's ControllerRefManager.ClaimObject as used by
// [EXT] kubeflow/common (called from tensorflow/tfjob_controller.go:288-289
// GetPodsForJob and the services twin): for every object listed with the
// job's selector --
//   * controllerRef == this job (uid):  keep it while the selector still
//     matches, otherwise RELEASE it (drop our ownerReference);
//   * controllerRef == someone else:    ignore;
//   * no controllerRef (orphan):        ADOPT it (add our controllerRef)
//     unless the job or the object is being deleted.
// The shell re-reads the job before adopting (RecheckDeletionTimestamp).
#include "core.h"

namespace toa {

static bool selector_matches(const Json& obj, const Json& selector) {
  const Json& labels = obj.path({"metadata", "labels"});
  for (const auto& kv : selector.fields())
    if (labels.get(kv.first).str() != kv.second.str()) return false;
  return true;
}

static const Json* controller_ref(const Json& obj) {
  for (const auto& r : obj.path({"metadata", "ownerReferences"}).items())
    if (r.get("controller").as_bool(false)) return &r;
  return nullptr;
}

Json claim_objects(const Json& job, const Json& objs) {
  const KindInfo& ki = kind_info(job_kind(job));
  const Json& md = job.get("metadata");
  const std::string uid = md.get("uid").str();
  const bool job_deleting = !md.get("deletionTimestamp").is_null();
  // the list selector: group-name + job-name (the labels every generation of
  // the reference's pods carries; controller-name is newer)
  const Json all = gen_labels(ki, md.get("name").str());
  Json selector = Json::object();
  selector.set(kLabelGroupName, all.get(kLabelGroupName));
  selector.set(kLabelJobName, all.get(kLabelJobName));
  Json claimed = Json::array(), adopt = Json::array(), release = Json::array();
  for (const auto& o : objs.items()) {
    const Json* ref = controller_ref(o);
    const bool matches = selector_matches(o, selector);
    if (ref != nullptr) {
      if (ref->get("uid").str() != uid) continue;  // owned by another controller
      if (matches) {
        claimed.push_back(o);
      } else if (!job_deleting) {
        release.push_back(o.path({"metadata", "name"}));
      }
      continue;
    }
    if (job_deleting || !matches || !o.path({"metadata", "deletionTimestamp"}).is_null()) continue;
    Json a = o;
    Json& omd = a["metadata"];
    Json owners = omd.get("ownerReferences").is_array() ? omd.get("ownerReferences") : Json::array();
    owners.push_back(owner_reference(job));
    omd.set("ownerReferences", owners);
    claimed.push_back(a);
    adopt.push_back(o.path({"metadata", "name"}));
  }
  Json res = Json::object();
  res.set("claimed", claimed);
  res.set("adopt", adopt);
  res.set("release", release);
  res.set("owner_reference", owner_reference(job));
  return res;
}

}  // namespace toa
