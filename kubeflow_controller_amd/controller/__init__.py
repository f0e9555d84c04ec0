"""TFJob controller: reconcile loop, helper, pod/service control, ref managers, updaters."""
from .control import (FakePodControl, FakeServiceControl, RealPodControl, RealServiceControl,
                      get_pod_from_template, validate_controller_ref)
from .controller import CONTROLLER_NAME, Controller
from .helper import Helper, claim_selector
from .ref import PodControllerRefManager, ServiceControllerRefManager
from .updater import DistributedUpdater, LocalUpdater
from .util import filter_pods, get_status, new_controller_ref
