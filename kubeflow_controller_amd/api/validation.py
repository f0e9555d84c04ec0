"""TFJob defaulting and validation.

The reference has neither: ``controller.go:311`` is a ``TODO: Check if the
TFJob is valid`` and a nil ``replicas`` panics at ``distributed.go:60`` even
though ``types.go:59`` documents "Default 1".  Here the store runs
``set_defaults`` + ``validate`` on create/update so the planner can rely on the
invariants the reference only assumed:

* every spec has a type in {PS, Worker, Local} and a template with >=1 container;
* ``replicas`` defaults to 1 and is >= 0;
* a ``Local`` job has exactly one spec (at ``Specs[0]``, ``checker.go:8-14``);
* a distributed job has exactly one Worker spec and at most one PS spec, at
  ``Specs[0]``/``Specs[1]`` (``distributed.go:198-206``).
"""
from __future__ import annotations

from typing import List

from . import v1alpha1
from .core import PodSpec, PodTemplateSpec


class ValidationError(ValueError):
    def __init__(self, errors: List[str]):
        super().__init__("; ".join(errors))
        self.errors = errors


def set_defaults(job: v1alpha1.TFJob) -> v1alpha1.TFJob:
    if not job.metadata.namespace:
        job.metadata.namespace = "default"
    for spec in job.spec.specs:
        if spec.replicas is None:
            spec.replicas = 1
        if spec.template is None:
            spec.template = PodTemplateSpec()
        if spec.template.spec is None:
            spec.template.spec = PodSpec()
        if spec.template.metadata.labels is None:
            spec.template.metadata.labels = {}
    return job


def validate(job: v1alpha1.TFJob) -> None:
    errs: List[str] = []
    if not job.metadata.name and not job.metadata.generateName:
        errs.append("metadata.name: required")
    specs = job.spec.specs
    if not specs:
        errs.append("spec.tfReplicaSpec: at least one replica spec is required")
    seen = {}
    for i, s in enumerate(specs):
        path = f"spec.tfReplicaSpec[{i}]"
        if s.tfReplicaType not in v1alpha1.REPLICA_TYPES:
            errs.append(f"{path}.tfReplicaType: must be one of {list(v1alpha1.REPLICA_TYPES)}, got {s.tfReplicaType!r}")
        if s.replicas is not None and s.replicas < 0:
            errs.append(f"{path}.replicas: must be >= 0")
        if s.template is None or not s.template.spec.containers:
            errs.append(f"{path}.template.spec.containers: at least one container is required")
        if s.tfReplicaType in seen:
            errs.append(f"{path}.tfReplicaType: duplicate {s.tfReplicaType} spec (also at [{seen[s.tfReplicaType]}])")
        seen.setdefault(s.tfReplicaType, i)
    types = [s.tfReplicaType for s in specs]
    if v1alpha1.LOCAL in types:
        if types[0] != v1alpha1.LOCAL or len(specs) != 1:
            errs.append("spec.tfReplicaSpec: a Local job has exactly one spec, of type Local, at index 0")
        elif specs[0].replicas not in (None, 1):
            errs.append("spec.tfReplicaSpec[0].replicas: a Local job runs exactly 1 replica")
    elif specs:
        if v1alpha1.WORKER not in types:
            errs.append("spec.tfReplicaSpec: a distributed job needs a Worker spec")
        if len(specs) > 2:
            errs.append("spec.tfReplicaSpec: a distributed job has at most a Worker and a PS spec")
    if errs:
        raise ValidationError(errs)
