# BioEngine datasets server (zarr-over-HTTP range reads + manifest registry); CPU only.
#   docker build -f docker/datasets.Dockerfile -t bioengine-datasets-amd .
#   docker run -v $DATA_DIR:/data -p 39527:39527 bioengine-datasets-amd
FROM python:3.11-slim

ENV PYTHONDONTWRITEBYTECODE=1 PYTHONUNBUFFERED=1 HOME=/home
WORKDIR /app
RUN apt-get update && apt-get install -y --no-install-recommends curl && rm -rf /var/lib/apt/lists/* \
    && python -m pip install --no-cache-dir fastapi uvicorn pyyaml numpy httpx aiohttp "zarr>=3"
COPY bioengine_worker_amd/__init__.py ./bioengine_worker_amd/__init__.py
COPY bioengine_worker_amd/datasets ./bioengine_worker_amd/datasets
COPY bioengine_worker_amd/utils ./bioengine_worker_amd/utils
EXPOSE 39527
CMD ["python", "-m", "bioengine_worker_amd.datasets", "--data-dir", "/data", "--server-ip", "0.0.0.0", "--server-port", "39527"]
