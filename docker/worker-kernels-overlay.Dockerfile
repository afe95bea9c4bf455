# Overlay: rebuild only the native libraries (HIP kernels + C++ runtime) and the Python package on
# top of a published worker image — the analog of the reference's Ray-version overlay
# (docker/worker-ray-overlay.Dockerfile there swaps Ray; here there is no Ray, and what changes
# between releases is the kernel library).
#   docker build -f docker/worker-kernels-overlay.Dockerfile \
#       --build-arg BASE_IMAGE=ghcr.io/aicell-lab/bioengine-worker-amd:0.1.0 -t bioengine-worker-amd:dev .
ARG BASE_IMAGE=bioengine-worker-amd:latest
FROM ${BASE_IMAGE}
WORKDIR /app
COPY csrc ./csrc
COPY tools ./tools
COPY bioengine_worker_amd ./bioengine_worker_amd
COPY bioengine ./bioengine
COPY apps ./apps
RUN python tools/build_native.py -j 8 && python -m pip install --no-cache-dir --no-deps --force-reinstall .
