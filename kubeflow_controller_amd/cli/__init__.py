"""Command-line entry points: ``kubeflow-controller`` and ``kfctl``."""
