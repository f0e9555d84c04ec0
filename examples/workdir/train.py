"""Generic replica entry point for the MI355X example TFJobs (ResNet-50, BERT-base,
Wide&Deep, MNIST): forwards its flags plus the controller's cluster-spec flags
(--worker_hosts/--ps_hosts/--job_name/--task_index) to the replica runtime."""
import sys

from kubeflow_controller_amd.trainer.replica import main

if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
