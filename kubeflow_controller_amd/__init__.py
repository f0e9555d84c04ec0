"""kubeflow_controller_amd — an MI355X-native TFJob controller and in-node training runtime.

Control plane (capabilities of gaocegege/kubeflow-controller):
  api/        TFJob v1alpha1 types (unchanged JSON contract), core objects, serde, validation
  store/      object store (apiserver/etcd/GC), REST server + client
  client/     clientset, informers/listers, event recorder
  native/     C++ workqueue + rate limiters, expectations, process launcher
  checker/    IsLocalJob
  planner/    local + distributed job planners, cluster spec / TF_CONFIG
  controller/ reconcile loop, helper, pod/service control, ref manager, updaters
  kubelet/    replica process supervisor + endpoint registry (one process per replica, GPU pinned)
  cli/        kubeflow-controller binary and kfctl client

Data plane (inside each replica):
  trainer/    replica runtime: cluster-spec parsing, role dispatch, trainer loop
  models/     MNIST softmax/MLP, ResNet-50, BERT-base, Wide&Deep
  ops/        hand-written CDNA4 HIP kernels (MFMA GEMM/conv, BN, softmax-xent, optimizers, embedding, ...)
  parallel/   RCCL data-parallel / parameter-server sharding over xGMI
"""
from .version import __version__  # noqa: F401
