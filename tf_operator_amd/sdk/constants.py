"""SDK constants (reference: sdk/python/kubeflow/tfjob/constants/constants.py:18-33)."""
import os

TFJOB_GROUP = "kubeflow.org"
TFJOB_KIND = "TFJob"
TFJOB_PLURAL = "tfjobs"
TFJOB_VERSION = os.environ.get("TFJOB_VERSION", "v1")
TFJOB_LOGLEVEL = os.environ.get("TFJOB_LOGLEVEL", "INFO").upper()
APISERVER_TIMEOUT = 120

TFJOB_GROUP_LABEL = "group-name"
TFJOB_NAME_LABEL = "job-name"
TFJOB_TYPE_LABEL = "replica-type"
TFJOB_INDEX_LABEL = "replica-index"
TFJOB_ROLE_LABEL = "job-role"

PLURALS = {"TFJob": "tfjobs", "PyTorchJob": "pytorchjobs", "MXJob": "mxjobs", "XGBoostJob": "xgboostjobs"}
