"""Training: Cellpose fine-tuning (single GPU and data-parallel over RCCL)."""
