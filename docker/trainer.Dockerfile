# Trainer image: PyTorch-ROCm + the gfx950 HIP kernel library + payloads.
# Build on a ROCm 7.x PyTorch base (hipcc cross-compiles gfx950 without a GPU).
ARG BASE=rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.10.0
FROM ${BASE}
WORKDIR /opt/tf-operator-amd
COPY csrc csrc
COPY tf_operator_amd tf_operator_amd
COPY pyproject.toml bench.py __graft_entry__.py ./
ENV PYTORCH_ROCM_ARCH=gfx950 PYTHONPATH=/opt/tf-operator-amd PYTHONUNBUFFERED=1 \
    HSA_ENABLE_IPC_MODE_LEGACY=0
RUN pip install --no-cache-dir pybind11 && python -m tf_operator_amd._build
# default payload: the Llama-3-8B data-parallel trainer (override in the job spec)
CMD ["python", "-m", "tf_operator_amd.examples.llama_train"]
