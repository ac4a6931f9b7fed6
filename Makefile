# Developer entry points (the reference's Makefile: build / test / manifests / images).
PY ?= python

.PHONY: build build-hip build-core crds test test-gpu bench e2e images clean

build:            ## gfx950 HIP kernels + C++ operator core
	$(PY) -m tf_operator_amd._build
build-hip:
	$(PY) -m tf_operator_amd._build --only hip
build-core:
	$(PY) -m tf_operator_amd._build --only core
crds:             ## regenerate manifests/base CRDs from tf_operator_amd/api/schema.py
	$(PY) -m tf_operator_amd.api.schema --out manifests/base
test: build       ## CPU tiers
	$(PY) -m pytest tests -q -m "not gpu"
test-gpu: build   ## kernel numerics (MI355X)
	$(PY) -m pytest tests -q -m gpu
bench: build      ## Llama-3-8B training step, one GPU
	$(PY) bench.py
e2e:              ## operator + kubelet + a job, no Kubernetes
	$(PY) -m tf_operator_amd.testing.cluster --apply manifests/examples/tfjob-dist-mnist.yaml --wait
images:
	docker build -f docker/operator.Dockerfile -t tf-operator-amd/training-operator:v0.1.0 .
	docker build -f docker/trainer.Dockerfile -t tf-operator-amd/trainer:v0.1.0 .
clean:
	rm -rf build tf_operator_amd/lib/*.so tf_operator_amd/core/*.so
