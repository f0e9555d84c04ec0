"""Local MNIST softmax regression (the reference's examples/workdir/mnist_softmax.py:
784->10 linear, GD lr 0.5, batch 100, 100,000 steps, ``step: i`` printed every step,
then the test accuracy) on the kubeflow_controller_amd runtime."""
import sys

from kubeflow_controller_amd.trainer.replica import main

if __name__ == "__main__":
    argv = ["--model", "mnist_softmax", "--optimizer", "sgd", "--learning_rate", "0.5", "--batch_size", "100",
            "--train_steps", "100000", "--log_every", "1"]
    sys.exit(main(argv + sys.argv[1:]))
