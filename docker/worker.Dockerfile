# BioEngine worker for AMD Instinct MI355X (gfx950).
#
# Base: the ROCm PyTorch image (ROCm 7.x runtime, hipcc, rocBLAS/hipBLASLt, RCCL, PyTorch-ROCm).
# The HIP kernel library is compiled for gfx950 at image build time (no GPU needed: hipcc
# cross-compiles), so containers start without a JIT step.
#
#   docker build -f docker/worker.Dockerfile -t bioengine-worker-amd:$(python -c "import tomllib;print(tomllib.load(open('pyproject.toml','rb'))['project']['version'])") .
#   docker run --device=/dev/kfd --device=/dev/dri --group-add video --group-add render \
#       --ipc=host --shm-size 8g -e HYPHA_TOKEN bioengine-worker-amd \
#       python -m bioengine_worker_amd.worker --mode single-machine --head-num-gpus 1
ARG ROCM_PYTORCH_IMAGE=rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.7.1
FROM ${ROCM_PYTORCH_IMAGE}

ENV PYTHONDONTWRITEBYTECODE=1 \
    PYTHONUNBUFFERED=1 \
    PYTORCH_ROCM_ARCH=gfx950 \
    BE_OFFLOAD_ARCH=gfx950 \
    # dmabuf IPC: RCCL / cross-process tensor sharing on current amdgpu drivers
    HSA_ENABLE_IPC_MODE_LEGACY=0 \
    HOME=/home/bioengine

WORKDIR /app

# Python dependencies first (layer cache); torch comes from the base image.
COPY pyproject.toml README.md ./
RUN python -m pip install --no-cache-dir numpy scipy pyyaml aiohttp cloudpickle msgpack click httpx \
        fastapi uvicorn "pydantic>=2" pillow safetensors pytest

COPY csrc ./csrc
COPY tools ./tools
COPY bioengine_worker_amd ./bioengine_worker_amd
COPY bioengine ./bioengine
COPY apps ./apps
COPY __graft_entry__.py bench.py ./

# Native libraries: libbe_hip.so (gfx950 HIP kernels) + libbe_runtime.so (C++ host runtime).
RUN python tools/build_native.py -j 8 \
    && python -m pip install --no-cache-dir --no-deps . \
    && python -c "import bioengine_worker_amd.ops._native as n; n.runtime(); print('native runtime ok')"

RUN mkdir -p /home/bioengine/.bioengine && chmod -R a+rwX /home/bioengine
ENV BIOENGINE_LOCAL_ARTIFACT_PATH=/app/apps

ENTRYPOINT []
CMD ["python", "-m", "bioengine_worker_amd.worker", "--mode", "single-machine"]
