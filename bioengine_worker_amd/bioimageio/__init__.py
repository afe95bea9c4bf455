"""BioImage.IO model support on MI355X (model-runner app).

bioimageio.core / bioimageio.spec are not part of this framework's dependency set; the subset of
their behaviour the model runner relies on is implemented here directly:

* :mod:`.spec` — RDF loading (format 0.4 and 0.5), format validation, axis / size / halo helpers.
* :mod:`.processing` — the bioimage.io pre/post-processing operators on GPU tensors.
* :mod:`.convert` — the MI355X graph pass: Conv2d(+BatchNorm)(+ReLU) chains become one fused NHWC
  MFMA conv kernel each, the network runs in bf16 channels-last.
* :mod:`.runner` — prediction pipeline: sample assembly, padding to valid sizes, tiled ("blocked")
  inference with halos, output cropping.
* :mod:`.testing` — ``test_model``: run the package's test inputs and compare with its test outputs.
* :mod:`.zoo` — model zoo access (hub artifacts or a local directory) and the on-disk model cache.
* :mod:`.package` — writes self-contained demo packages (used offline, by tests and by the bench).
"""
