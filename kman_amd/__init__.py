"""kman_amd — MI355X (gfx950) k-mer extract / sort / join engine.

Drop-in for the k-mer path of ggirelli/kman (package ``kmermaid`` 1.0.0): the
``kmer`` CLI and the FastaBatcher / Batch / Crawler / KJoiner surface are
kept, the per-base and per-k-mer work runs in HIP kernels behind the C ABI of
include/kman.h (libkman.so, loaded by ``_native``).
"""

__version__ = "0.1.0"

from . import phases as _phases  # noqa: E402

_phases.mark("interpreter+import")

__all__ = ["__version__", "batch", "batcher", "engine", "io", "join", "seq", "source"]
