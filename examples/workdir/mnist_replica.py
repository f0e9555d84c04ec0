"""Distributed MNIST (the reference's examples/workdir/mnist_replica.py: 784->100 ReLU->10,
Adam lr 0.01, batch 100, 200 global steps, minimising the summed cross-entropy of
clipped probabilities) on the kubeflow_controller_amd runtime.
Takes the controller's --worker_hosts/--ps_hosts/--job_name/--task_index flags."""
import sys

from kubeflow_controller_amd.trainer.replica import main

if __name__ == "__main__":
    argv = ["--model", "mnist_mlp", "--optimizer", "adam", "--learning_rate", "0.01", "--batch_size", "100",
            "--train_steps", "200", "--hidden_units", "100", "--loss", "sum_clipped", "--log_every", "10"]
    sys.exit(main(argv + sys.argv[1:]))
