"""``python -m kubeflow_controller_amd`` == the ``kubeflow-controller`` binary."""
import sys

from .cli.controller_main import main

sys.exit(main())
