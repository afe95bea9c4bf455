"""Electron-microscopy mitochondria analysis (fibsem-mito-analysis app; SURVEY.md §2.2 row 27,
§2.5 K14/K15): tiled inference with Gaussian-blended stitching, GPU post-processing (size filter,
disk closing, exact EDT, peak detection), marker watershed (C++ runtime) and regionprops."""
