"""Python SDK: TFJobClient + typed models (reference: sdk/python/kubeflow/tfjob)."""
from .models import (V1ElasticPolicy, V1ElasticStatus, V1JobCondition, V1JobStatus, V1ObjectMeta, V1ReplicaSpec,  # noqa: F401
                     V1ReplicaStatus, V1RunPolicy, V1SchedulingPolicy, V1TFJob, V1TFJobList, V1TFJobSpec,
                     container, pod_template)
from .tf_job_client import TFJobClient  # noqa: F401
