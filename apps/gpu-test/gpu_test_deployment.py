"""GPU sanity check: device visibility, rocm-smi, and one HIP kernel launch through torch."""
import os
import shutil
import subprocess

from hypha_rpc.utils.schema import schema_method
from ray import serve


@serve.deployment(ray_actor_options={"num_cpus": 1, "num_gpus": 1})
class GpuTest:
    @schema_method
    async def ping(self) -> str:
        """Liveness."""
        return "pong"

    @schema_method
    async def gpu_info(self) -> dict:
        """Visible devices, rocm-smi product listing and a matmul on the replica's GPU."""
        info = {"HIP_VISIBLE_DEVICES": os.environ.get("HIP_VISIBLE_DEVICES"),
                "ROCR_VISIBLE_DEVICES": os.environ.get("ROCR_VISIBLE_DEVICES")}
        smi = shutil.which("rocm-smi") or "/opt/rocm/bin/rocm-smi"
        try:
            info["rocm_smi"] = subprocess.run([smi, "--showproductname"], capture_output=True, text=True,
                                              timeout=20).stdout
        except Exception as e:  # noqa: BLE001
            info["rocm_smi"] = f"unavailable: {e}"
        try:
            import torch

            info["device_count"] = torch.cuda.device_count()
            if torch.cuda.is_available():
                p = torch.cuda.get_device_properties(0)
                a = torch.randn(256, 256, device="cuda")
                info.update(device_name=p.name, arch=getattr(p, "gcnArchName", None),
                            total_memory_gb=round(p.total_memory / 1024 ** 3, 1),
                            matmul_ok=bool(torch.isfinite(a @ a).all().item()))
        except Exception as e:  # noqa: BLE001
            info["torch_error"] = str(e)
        return info
