"""SDK helpers and constants (reference: sdk/python/kubeflow/tfjob/utils/utils.py:19-74,
constants/constants.py:18-33): label sets, selectors, namespace resolution."""
from tf_operator_amd.sdk import V1ObjectMeta, V1TFJob, constants, utils


def test_constants_match_reference():
    assert (constants.TFJOB_GROUP, constants.TFJOB_KIND, constants.TFJOB_PLURAL) == ("kubeflow.org", "TFJob", "tfjobs")
    assert constants.TFJOB_VERSION == "v1"
    assert (constants.TFJOB_NAME_LABEL, constants.TFJOB_TYPE_LABEL, constants.TFJOB_INDEX_LABEL) == (
        "job-name", "replica-type", "replica-index")


def test_labels_and_selector():
    assert utils.get_labels("j") == {"group-name": "kubeflow.org", "job-name": "j"}
    lab = utils.get_labels("j", master=True, replica_type="Worker", replica_index=2)
    assert lab[constants.TFJOB_ROLE_LABEL] == "master"
    assert lab["replica-type"] == "worker" and lab["replica-index"] == "2"
    assert utils.to_selector({"a": "1", "b": "x"}) == "a=1,b=x"


def test_namespace_resolution(monkeypatch, tmp_path):
    monkeypatch.setattr(utils, "SA_DIR", str(tmp_path / "absent"))
    assert not utils.is_running_in_k8s() and utils.get_default_target_namespace() == "default"
    assert utils.set_tfjob_namespace({"metadata": {"namespace": "team-a"}}) == "team-a"
    assert utils.set_tfjob_namespace({"metadata": {}}) == "default"
    job = V1TFJob(metadata=V1ObjectMeta(name="x", namespace="team-b"))
    assert utils.set_tfjob_namespace(job) == "team-b"
    sa = tmp_path / "sa"
    (sa / "serviceaccount").mkdir(parents=True)
    (sa / "serviceaccount" / "namespace").write_text("kubeflow\n")
    monkeypatch.setattr(utils, "SA_DIR", str(sa))
    assert utils.is_running_in_k8s() and utils.get_default_target_namespace() == "kubeflow"
