# Operator image: the C++17 core (pybind11) + asyncio shell.  No GPU libraries.
FROM python:3.10-slim AS build
RUN apt-get update && apt-get install -y --no-install-recommends g++ && rm -rf /var/lib/apt/lists/*
WORKDIR /src
COPY csrc/core csrc/core
COPY tf_operator_amd tf_operator_amd
COPY pyproject.toml .
RUN pip install --no-cache-dir pybind11 aiohttp prometheus_client pyyaml numpy \
 && python -m tf_operator_amd._build --only core

FROM python:3.10-slim
RUN pip install --no-cache-dir aiohttp prometheus_client pyyaml numpy
WORKDIR /opt/tf-operator-amd
COPY --from=build /src/tf_operator_amd tf_operator_amd
ENV PYTHONPATH=/opt/tf-operator-amd PYTHONUNBUFFERED=1
USER 65532:65532
ENTRYPOINT ["python", "-m", "tf_operator_amd.operator.main"]
