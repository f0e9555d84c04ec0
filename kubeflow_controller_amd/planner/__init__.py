"""TF job planners — "what to create" (reference ``pkg/tensorflow``)."""
from .distributed import PORT_NAME, TF_CONFIG_ENV, WORKER_PORT, DistributedJob
from .local import EXPECTED_LOCAL_WORKER_NUMBER, LocalJob, job_labels
from .types import Action, Event
from .util import generate_name, generate_runtime_id
