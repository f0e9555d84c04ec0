"""Client machinery: clientset, informers/listers, events, workqueue/expectations."""
from .clientset import Clientset, ResourceClient
from .events import NORMAL, WARNING, EventBroadcaster, EventRecorder, FakeRecorder
from .informer import Lister, SharedInformer, SharedInformerFactory
