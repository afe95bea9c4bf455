"""Cell morphology search: GPU pre-processing, nucleus crops, DINOv2 embedding, vector index,
2-D projection and the ingestion pipeline behind the cell-image-search app
(reference apps/cell-image-search/)."""
