"""TFJob API (``kubeflow.caicloud.io/v1alpha1``) plus the core objects the
controller derives from it.  See ``v1alpha1.py`` for the contract."""
from . import core, meta, v1alpha1
from .core import Container, Event, Pod, PodSpec, PodTemplateSpec, Service, ServicePort, ServiceSpec
from .meta import ObjectMeta, OwnerReference, generate_name, get_controller_of, key_of, split_key
from .serde import dump_json, dump_yaml, envsubst, load_file, load_objects
from .v1alpha1 import TFJob, TFJobSpec, TFJobStatus, TFReplicaSpec, TFReplicaStatus
from .validation import ValidationError, set_defaults, validate
