# Build / test / bench entry points (reference: Makefile:1-34 — `make build`,
# `make test`, `make clean`; version metadata injected at build time).
#
#   make build       compile the C++ runtime, the comm helpers and every HIP kernel for gfx950 (in-tree)
#   make test        CPU test suite (API, store, controller, planner, e2e TFJobs, gloo DP / PS / async PS)
#   make sanitize   runtime core self-test under ASan+UBSan and TSan (host code only)
#   make test-gpu    GPU test suite (every HIP kernel vs a PyTorch fp32 reference, model steps) — on an MI355X
#   make bench       headline benchmark (ResNet-50 training images/s, 1 GPU; GPUS=N for torchrun)
#   make version     version / git SHA / runtime
#   make clean       remove built artefacts

PYTHON   ?= python3
ARCH     ?= gfx950
GPUS     ?= 1
STEPS    ?= 20
WARMUP   ?= 5
GIT_SHA  := $(shell git rev-parse --short HEAD 2>/dev/null || echo unknown)

export PYTORCH_ROCM_ARCH := $(ARCH)
export KFA_GIT_SHA := $(GIT_SHA)

.PHONY: build sanitize test test-gpu bench version clean

build:
	$(PYTHON) -m kubeflow_controller_amd._build --force

test:
	$(PYTHON) -m pytest tests/ -x -q -m "not gpu"

sanitize:
	$(PYTHON) -m kubeflow_controller_amd._build --sanitize

test-gpu:
	$(PYTHON) -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread

bench:
ifeq ($(GPUS),1)
	$(PYTHON) bench.py --gpus 1 --steps $(STEPS) --warmup $(WARMUP)
else
	$(PYTHON) -m torch.distributed.run --nnodes=1 --nproc-per-node $(GPUS) --master-addr 127.0.0.1 \
		--master-port 29500 bench.py --gpus $(GPUS) --steps $(STEPS) --warmup $(WARMUP)
endif

version:
	$(PYTHON) bin/kubeflow-controller -version

clean:
	rm -rf build
	find kubeflow_controller_amd -name "*.so" -delete -o -name "*.so.stamp" -delete
