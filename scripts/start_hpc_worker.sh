#!/bin/bash
# Start the BioEngine head worker on an HPC login/head node inside Apptainer (or Singularity), with
# SLURM worker jobs for the GPU nodes (MI355X: ROCm device pass-through via `--rocm`).
#
#   scripts/start_hpc_worker.sh [worker args...]
#       --image PATH.sif|docker://URI   container image (default: the bioengine-worker-amd image of this version)
#       --workspace-dir DIR             worker state on the shared filesystem (default ~/.bioengine)
#       --debug                         bind the current checkout to /app (run local code)
#   every other argument is passed to `python -m bioengine_worker_amd.worker` unchanged.
#
# The head worker submits `bioengine-worker` SLURM jobs that run the node agent
# (python -m bioengine_worker_amd.cluster.node_agent) in the same image; on exit this script
# cancels the jobs it left behind.  Reference behaviour: scripts/start_hpc_worker.sh of
# aicell-lab/bioengine-worker (Ray head + `--nv`), re-done for the native runtime.
set -uo pipefail

here="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
root="$(dirname "$here")"

version="$(sed -nE 's/^version[[:space:]]*=[[:space:]]*"([^"]+)".*/\1/p' "$root/pyproject.toml" 2>/dev/null | head -1)"
version="${version:-latest}"

if command -v apptainer >/dev/null 2>&1; then runner=apptainer
elif command -v singularity >/dev/null 2>&1; then runner=singularity
else echo "error: apptainer or singularity is required" >&2; exit 1
fi

# ---- split our options from the worker's -------------------------------------------------------
image="docker://ghcr.io/aicell-lab/bioengine-worker-amd:${version}"
workspace="${HOME}/.bioengine"
debug=0
passthrough=()
while [[ $# -gt 0 ]]; do
    case "$1" in
        --image) image="$2"; shift 2 ;;
        --image=*) image="${1#*=}"; shift ;;
        --workspace-dir) workspace="$2"; shift 2 ;;
        --workspace-dir=*) workspace="${1#*=}"; shift ;;
        --debug) debug=1; passthrough+=("--debug"); shift ;;
        --mode|--mode=*)
            m="${1#--mode=}"; [[ "$1" == "--mode" ]] && { m="$2"; shift; }
            shift
            if [[ "$m" != "slurm" ]]; then
                echo "error: this launcher runs --mode slurm; run the container directly for '$m'" >&2; exit 1
            fi ;;
        *) passthrough+=("$1"); shift ;;
    esac
done

if [[ "$image" == *.sif ]]; then
    image="$(realpath "$image")"
    [[ -f "$image" ]] || { echo "error: image $image not found" >&2; exit 1; }
elif [[ "$image" != docker://* ]]; then
    image="docker://$image"
fi

mkdir -p "$workspace"
workspace="$(realpath "$workspace")"
export APPTAINER_CACHEDIR="${APPTAINER_CACHEDIR:-$workspace/images}"
export SINGULARITY_CACHEDIR="$APPTAINER_CACHEDIR"
mkdir -p "$APPTAINER_CACHEDIR"

# ---- bind mounts: SLURM client + munge, workspace, optional source checkout -----------------------
binds=()
bind_if() { [[ -e "$1" ]] && binds+=("--bind" "$1${2:+:$2}"); return 0; }
for tool in sbatch squeue scancel sinfo; do
    p="$(command -v "$tool" 2>/dev/null)" && bind_if "$p"
done
for p in /etc/slurm /etc/munge /var/run/munge /var/lib/munge /usr/lib64/slurm /etc/hosts /etc/passwd /etc/group \
         /etc/localtime; do
    bind_if "$p"
done
for lib in /usr/lib64/libmunge.so*; do bind_if "$lib"; done
binds+=("--bind" "$workspace:$workspace")
workdir=/app
if [[ $debug -eq 1 ]]; then
    binds+=("--bind" "$root:/app")
    echo "debug: running the checkout at $root"
fi

# ---- environment ---------------------------------------------------------------------------------
if [[ -f "$PWD/.env" ]]; then set -a; source "$PWD/.env"; set +a; fi
envs=("--env" "HSA_ENABLE_IPC_MODE_LEGACY=0" "--env" "USER=${USER:-bioengine}")
[[ -n "${HYPHA_TOKEN:-}" ]] && envs+=("--env" "HYPHA_TOKEN=$HYPHA_TOKEN")

cleanup() {
    # Worker jobs are named "bioengine-worker" (bioengine_worker_amd/cluster/slurm.py JOB_NAME).
    if command -v squeue >/dev/null 2>&1; then
        ids="$(squeue -u "${USER:-$(id -un)}" -n bioengine-worker -h -o %i 2>/dev/null)"
        if [[ -n "$ids" ]]; then
            echo "cancelling leftover BioEngine worker jobs: $ids"
            # shellcheck disable=SC2086
            scancel $ids
        fi
    fi
}
trap cleanup EXIT

"$runner" exec --rocm --cleanenv --pwd "$workdir" "${envs[@]}" "${binds[@]}" "$image" \
    python -m bioengine_worker_amd.worker --mode slurm --workspace-dir "$workspace" --image "$image" \
    "${passthrough[@]}"
