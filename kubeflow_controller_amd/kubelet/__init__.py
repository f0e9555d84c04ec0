"""Single-node kubelet: replica process supervisor + endpoint controller."""
from .endpoints import EndpointController, PortAllocator, service_host_map
from .supervisor import Supervisor, detect_gpus
