"""File plumbing around the k-mer path (kmermaid/io.py)."""

from __future__ import annotations

import gzip
import os
import tempfile
from typing import List

import numpy as np

from .batch import Batch


def set_tempdir(path: str, create: bool = True) -> None:
    """io.py:18-32."""
    if not os.path.isdir(path):
        if create:
            os.makedirs(path, exist_ok=True)
        else:
            raise AssertionError(f"folder not found: {path}")
    tempfile.tempdir = path


def input_file_exists(path: str) -> None:
    """io.py:35-43."""
    if not os.path.isfile(path):
        raise AssertionError(f"input file not found: {path}")


def batch_files(batches: List[Batch]):
    """(batch, sorted FASTA bytes) of every non-empty device batch.

    All batches of one source are sorted in ONE device pass: the keys are
    tagged with their batch index above the 2k key bits (kman_tag_batches) so
    a single stable radix sort orders every batch on its own (batch.py:156-168
    for each batch; ties keep stream order like Timsort)."""
    from .source import download_sorted

    by_src = {}
    for b in batches:
        if b.current_size and b.on_device:
            by_src.setdefault(id(b.source), (b.source, []))[1].append(b)
    for src, bs in by_src.values():
        lo = min(b.stream_range[0] for b in bs)
        hi = max(b.stream_range[1] for b in bs)
        contiguous = sum(b.current_size for b in bs) == hi - lo
        uniform = len({b.size for b in bs}) == 1 and all(b.stream_range[0] % bs[0].size == 0 for b in bs)
        if contiguous and uniform and hasattr(src, "parsed") and hasattr(src, "rc"):
            keys, pos = download_sorted(src, lo, hi, True, per_batch=bs[0].size)
            for b in bs:
                s, e = b.stream_range
                yield b, src.format_fasta(keys[s - lo : e - lo], pos[s - lo : e - lo])
        else:
            for b in bs:
                yield b, b.fasta_bytes()
    for b in batches:
        if b.current_size and not b.on_device and b.is_written and os.path.isfile(b.tmp):
            with open(b.tmp, "rb") as fh:
                yield b, fh.read()


def copy_batches(batches: List[Batch], output_path: str, compress: bool = False) -> None:
    """Write every batch's sorted FASTA into ``output_path`` as
    ``<basename(batch.tmp)>`` (``.gz`` with ``compress``) — io.py:46-71.  The
    bytes come straight from the device; no temp copy is made first."""
    for b, data in batch_files(batches):
        name = os.path.basename(b.tmp)
        if compress:
            with gzip.open(os.path.join(output_path, name + ".gz"), "wb") as OH:
                OH.write(data)
        else:
            with open(os.path.join(output_path, name), "wb") as OH:
                OH.write(data)


__all__ = ["set_tempdir", "input_file_exists", "copy_batches", "batch_files", "np"]
