"""dlq_amd -- MI355X-native int8 inference path of yeontachi/DLQ's
ResNet-18 kernel lab and MNIST FC GEMM.

Submodules:
  lib      ctypes binding of libdlq.so (the C ABI in include/dlq.h)
  ops      per-layer operators (reference names, int8 NHWC)
  models   ResNet18Int8 / MLPInt8 engines + the fp32 torch definitions used
           for calibration and the CPU baseline
  quant    activation-scale calibration (the int8 "quant block")
"""
__version__ = "0.1.0"
