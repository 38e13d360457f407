"""gpusdr: host-side Python package over libgpusdrpipeline.so (MI355X / gfx950).

The product is the C-ABI shared library (include/gsdr/*.h kernels, include/gpusdrpipeline/*
filter graph). This package is the Python plumbing the tests and bench use: tensor wrappers
(ops), time-sharding over torch.distributed (shard) and the path helpers.
"""
import os

REPO_ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
PKG_ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
