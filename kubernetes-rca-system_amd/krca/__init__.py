"""krca — MI355X-native numeric core for Kubernetes root-cause analysis.

Host side (this package, Python) mirrors the reference's agent API; the numeric hot path runs in
``libkrca.so`` (hand-written HIP for gfx950, C-ABI in ``include/krca.h``), reached through
:mod:`krca.native`.  There is no CPU fallback on the product path.
"""
__version__ = "0.1.0"
