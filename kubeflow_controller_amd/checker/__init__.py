"""Job-kind checker (reference ``pkg/checker/checker.go:8-14``)."""
from ..api import v1alpha1


def is_local_job(tfjob: v1alpha1.TFJob) -> bool:
    """True iff ``Specs[0].TFReplicaType == "Local"``."""
    specs = tfjob.spec.specs
    return bool(specs) and specs[0].tfReplicaType == v1alpha1.LOCAL


IsLocalJob = is_local_job
