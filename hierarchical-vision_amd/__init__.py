"""MI355X-native SwinV2 + taxonomy-loss training hot path (drop-in for the
model/loss layer of samuelstevens/hierarchical-vision).

Modules mirror the reference files they replace:
  swinv2.py      <- swinv2.py      (SwinTransformerV2 & friends, same state-dict keys)
  hierarchy.py   <- hierarchy.py   (taxonomy parsing, MultitaskHead, losses incl. HXE)
  models.py      <- models.py      (build_model / build_composer_model / Model)
  algorithmic.py <- algorithmic.py (LabelSmoothing for list outputs)
  configs.py     <- configs.py     (structured config schema)
  ddp.py            RCCL gradient all-reduce, bucketed, overlapped with backward
  ops.py            autograd Functions over the C ABI of libhvk.so
  _lib.py           ctypes binding of libhvk.so (include/hvk.h)
Import as ``hvamd`` (see ../hvamd.py).
"""
__version__ = "0.1.0"
