"""ctypes binding of libkman.so (the C ABI declared in include/kman.h).

This module is the only place Python touches the native library.  Loading is
strict: if the in-tree ``kman_amd/lib/libkman.so`` is missing the import of any
engine entry point raises — there is no CPU fallback on the product path.

Error mapping follows the reference: argument errors the reference raises as
``AssertionError`` (k <= 1, empty FASTA, ...) stay ``AssertionError``; device
and runtime failures become ``RuntimeError``.
"""

from __future__ import annotations

import ctypes
import os
import threading
from ctypes import POINTER, c_char_p, c_int, c_size_t, c_uint32, c_uint64, c_void_p

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KMAN_LIB", os.path.join(HERE, "lib", "libkman.so"))

KMAN_OK = 0
KMAN_EINVAL = -1
KMAN_EHIP = -2
KMAN_ENOMEM = -3
KMAN_EFORMAT = -4
KMAN_ETIMEOUT = -5
KMAN_ECOMM = -6
KMAN_ECAP = -7
KMAN_EFALLBACK = -8
KMAN_EPARTIAL = -9

KMAN_RC = 1
KMAN_WANT_POS = 2
KMAN_CANONICAL = 4
KMAN_MIXED = 8
KMAN_ONCE = 16
KMAN_ROOMY = 32
KMAN_FINISH_SORT = 0
KMAN_FINISH_COUNT = 1
KMAN_FINISH_UNIQ = 2
KMAN_PARSE_IN_RECORD = 1


def KMAN_HIST_LO(b: int) -> int:
    return (int(b) & 0x7F) << 8


class ParseInfo(ctypes.Structure):
    _fields_ = [("n_bases", c_uint64), ("n_records", c_uint64)]


class Run(ctypes.Structure):
    """kman_run: one sorted run for kman_merge_runs."""
    _fields_ = [("keys", c_void_p), ("vals", c_void_p), ("n", c_uint64)]


# name -> (restype, argtypes); every symbol include/kman.h declares
SIGNATURES = {
    "kman_abi_version": (c_int, []),
    "kman_device_count": (c_int, [POINTER(c_int)]),
    "kman_create": (c_int, [c_int, POINTER(c_void_p)]),
    "kman_destroy": (None, [c_void_p]),
    "kman_last_error": (c_char_p, [c_void_p]),
    "kman_sync": (c_int, [c_void_p]),
    "kman_malloc": (c_int, [c_void_p, POINTER(c_void_p), c_size_t]),
    "kman_format_count_dev": (
        c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_uint64, c_uint32, c_void_p, c_size_t, POINTER(c_size_t)],
    ),
    "kman_format_uniq_dev": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_uint32, c_uint64, c_uint32, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p,
         c_size_t, POINTER(c_size_t)],
    ),
    "kman_mem_info": (c_int, [c_void_p, POINTER(c_size_t), POINTER(c_size_t)]),
    "kman_free": (c_int, [c_void_p, c_void_p]),
    "kman_host_alloc": (c_int, [c_void_p, POINTER(c_void_p), c_size_t]),
    "kman_host_free": (c_int, [c_void_p, c_void_p]),
    "kman_memcpy_h2d": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
    "kman_memcpy_d2h": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
    "kman_memset": (c_int, [c_void_p, c_void_p, c_int, c_size_t]),
    "kman_timing_enable": (c_int, [c_void_p, c_int]),
    "kman_timing_query": (c_int, [c_void_p, c_char_p, POINTER(c_uint64), POINTER(ctypes.c_double)]),
    "kman_parse_fasta": (
        c_int,
        [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_uint64, POINTER(ParseInfo)],
    ),
    "kman_count_kmers": (c_int, [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, POINTER(c_uint64)]),
    "kman_extract": (
        c_int,
        [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, c_void_p, c_void_p, c_uint32, c_uint64, c_void_p,
         POINTER(c_uint64)],
    ),
    "kman_extract_range": (
        c_int,
        [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, c_uint64, c_uint64, c_void_p, c_void_p, c_uint32, c_uint64,
         c_void_p, POINTER(c_uint64)],
    ),
    "kman_kmer_prefix_hist": (c_int, [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, c_void_p, POINTER(c_uint64)]),
    "kman_sort_plan": (c_int, [c_uint32, POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32)]),
    "kman_sort": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint32, c_uint64, c_uint32, c_void_p, POINTER(c_int)],
    ),
    "kman_sort_plan_range": (
        c_int, [c_uint32, c_uint32, POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32)]),
    "kman_sort_range": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint32, c_uint64, c_uint32, c_uint32, c_void_p,
         POINTER(c_int)],
    ),
    "kman_split_bits": (c_int, [c_uint64, c_uint32, POINTER(c_uint32)]),
    "kman_extract_sorted": (
        c_int,
        [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p,
         c_uint32, c_uint64, POINTER(c_uint64), POINTER(c_int)],
    ),
    "kman_finish": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint32, c_uint64, c_uint32, c_uint32, c_int,
         c_void_p, c_void_p, c_uint32, POINTER(c_uint64)],
    ),
    "kman_groups_plan": (c_int, [c_uint64, c_uint32, c_uint32, c_int, POINTER(c_uint64)]),
    "kman_groups": (
        c_int,
        [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, c_int, c_void_p, c_uint64, c_void_p, c_void_p, c_uint32,
         POINTER(c_uint64), POINTER(c_uint64)],
    ),
    "kman_groups_begin": (
        c_int,
        [c_void_p, c_uint64, c_uint32, c_uint32, c_int, c_void_p, c_uint64, POINTER(c_uint32), POINTER(c_uint64)],
    ),
    "kman_groups_extract": (
        c_int,
        [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, c_int, c_void_p, c_uint64, c_uint32],
    ),
    "kman_groups_end": (
        c_int,
        [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, c_int, c_void_p, c_uint64, c_void_p, c_void_p, c_uint32,
         POINTER(c_uint64), POINTER(c_uint64)],
    ),
    "kman_dshard_plan": (c_int, [c_uint64, c_uint64, c_uint32, c_uint32, c_int]),
    "kman_dshard_hist": (c_int, [c_void_p, c_void_p, c_uint64, c_uint64, c_uint32, c_uint32, c_int, c_void_p, c_void_p]),
    "kman_dshard_extract": (
        c_int, [c_void_p, c_void_p, c_uint64, c_uint64, c_uint32, c_uint32, c_int, c_void_p, c_void_p, c_void_p],
    ),
    "kman_dround_plan": (
        c_int, [c_uint32, c_uint32, c_int, c_uint32, c_uint64, c_uint32, c_void_p, POINTER(c_uint64), POINTER(c_uint64)],
    ),
    "kman_dround_finish": (
        c_int,
        [c_void_p, c_void_p, c_uint32, c_uint32, c_int, c_uint32, c_uint64, c_uint32, c_uint32, c_void_p, c_void_p,
         c_uint64, c_void_p, c_uint64, c_void_p, c_void_p, c_uint32, POINTER(c_uint64)],
    ),
    "kman_dround_failed": (c_int, [c_void_p, c_void_p, c_uint64, POINTER(c_uint64)]),
    "kman_dround_heavy": (c_int, [c_void_p, POINTER(c_uint32)]),
    "kman_dround_left": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, POINTER(c_uint64)]),
    "kman_dround_heavy_fix": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_uint64]),
    "kman_extract_marked": (
        c_int,
        [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, c_void_p, c_uint32, c_uint32, c_void_p, c_void_p, c_uint32,
         c_uint64, POINTER(c_uint64)],
    ),
    "kman_count_hist": (c_int, [c_void_p, c_void_p, c_uint32, c_uint64, c_void_p, c_uint32]),
    "kman_rle_count": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_uint32, POINTER(c_uint64)]),
    "kman_rle_uniq": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_uint32, c_uint64, c_void_p, c_void_p, POINTER(c_uint64)],
    ),
    "kman_comm_unique_id": (c_int, [c_void_p]),
    "kman_comm_init": (c_int, [c_void_p, c_void_p, c_int, c_int]),
    "kman_comm_count": (c_int, [c_void_p, c_void_p, c_void_p]),
    "kman_comm_destroy": (c_int, [c_void_p]),
    "kman_prefix_hist": (c_int, [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, c_void_p]),
    "kman_allreduce_u64": (c_int, [c_void_p, c_void_p, c_uint64]),
    "kman_allgather_u64": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64]),
    "kman_alltoallv": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint32]),
    "kman_alltoallv_async": (
        c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint32, c_int],
    ),
    "kman_comm_wait": (c_int, [c_void_p, c_int]),
    "kman_partition": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint32, c_uint64, c_void_p, c_uint32, c_uint32,
         c_void_p],
    ),
    "kman_tag_batches": (c_int, [c_void_p, c_void_p, c_uint64, c_uint32, c_uint64, c_uint64]),
    "kman_or_u64": (c_int, [c_void_p, c_void_p, c_uint64, c_uint64]),
    "kman_widen_u32": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_uint64]),
    "kman_memcpy_d2d": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
    "kman_extract_wide": (
        c_int, [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, c_void_p, c_void_p, c_void_p, c_uint32, c_uint64,
                POINTER(c_uint64)],
    ),
    "kman_iota_u64": (c_int, [c_void_p, c_void_p, c_uint64]),
    "kman_gather": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_uint32]),
    "kman_rle_wide": (
        c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_uint32, c_uint64, c_void_p, c_void_p, c_void_p,
                POINTER(c_uint64)],
    ),
    "kman_format_count_wide": (
        c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_uint64, c_uint32, c_void_p, c_size_t, POINTER(c_size_t),
                c_int],
    ),
    "kman_format_uniq_wide": (
        c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_uint64, c_uint32, c_void_p, c_void_p, c_void_p, c_uint64,
                c_void_p, c_size_t, POINTER(c_size_t), c_int],
    ),
    "kman_format_count_wide_dev": (
        c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint32, c_uint64, c_uint32, c_void_p, c_size_t,
                POINTER(c_size_t)],
    ),
    "kman_format_uniq_wide_dev": (
        c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint32, c_uint64, c_uint32, c_void_p, c_void_p, c_void_p,
                c_uint64, c_void_p, c_size_t, POINTER(c_size_t)],
    ),
    "kman_format_uniq_mixed": (
        c_int, [c_void_p, c_void_p, c_uint64, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p,
                c_size_t, POINTER(c_size_t), c_int],
    ),
    "kman_extract_words": (
        c_int, [c_void_p, c_void_p, c_uint64, c_uint32, c_uint32, c_void_p, c_uint64, c_void_p, c_uint32, c_uint64,
                POINTER(c_uint64)],
    ),
    "kman_rle_words": (
        c_int, [c_void_p, c_int, c_void_p, c_uint32, c_uint64, c_void_p, c_uint32, c_uint64, c_void_p, c_uint64,
                c_void_p, c_uint32, POINTER(c_uint64)],
    ),
    "kman_batch_tags": (c_int, [c_void_p, c_void_p, c_uint64, c_uint64, c_uint64, c_void_p]),
    "kman_format_count_words": (
        c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_uint64, c_uint32, c_void_p, c_size_t, POINTER(c_size_t),
                c_int],
    ),
    "kman_format_uniq_words": (
        c_int, [c_void_p, c_uint64, c_void_p, c_uint32, c_uint64, c_uint32, c_void_p, c_void_p, c_void_p, c_uint64,
                c_void_p, c_size_t, POINTER(c_size_t), c_int],
    ),
    "kman_format_uniq_mixed_words": (
        c_int, [c_void_p, c_uint64, c_void_p, c_uint64, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_uint64,
                c_void_p, c_size_t, POINTER(c_size_t), c_int],
    ),
    "kman_format_count_words_dev": (
        c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_uint32, c_uint64, c_uint32, c_void_p, c_size_t,
                POINTER(c_size_t)],
    ),
    "kman_format_uniq_words_dev": (
        c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_uint32, c_uint64, c_uint32, c_void_p, c_void_p, c_void_p,
                c_uint64, c_void_p, c_size_t, POINTER(c_size_t)],
    ),
    "kman_merge_runs": (c_int, [c_void_p, c_void_p, c_int, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "kman_count_descents": (c_int, [c_void_p, c_void_p, c_uint64, POINTER(c_uint64)]),
    "kman_row_digest": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_uint64, c_uint64, POINTER(c_uint64)]),
    "kman_format_vector": (c_int, [c_void_p, c_uint64, c_uint64, c_void_p, c_size_t, POINTER(c_size_t), c_int]),
    "kman_vec_fill": (
        c_int,
        [c_void_p, c_void_p, c_void_p, c_uint32, c_uint64, c_int, c_void_p, c_uint32, c_void_p, c_void_p, c_uint64,
         c_void_p],
    ),
    "kman_rebase_pos": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_uint32]),
    "kman_synth_fasta": (c_int, [c_void_p, c_void_p, c_uint64, c_uint64, c_uint64, c_void_p, c_uint32, c_uint32]),
    "kman_copy_h2d_async": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_int]),
    "kman_copy_wait": (c_int, [c_void_p, c_int]),
    "kman_copy_d2h_async": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_int]),
    "kman_copy_d2h_wait": (c_int, [c_void_p, c_int]),
    "kman_copy_sync": (c_int, [c_void_p]),
    "kman_parse_fasta_at": (
        c_int, [c_void_p, c_void_p, c_uint64, c_uint32, c_void_p, c_uint64, c_void_p, c_void_p, c_uint64, c_void_p],
    ),
    "kman_format_count": (
        c_int,
        [c_void_p, c_void_p, c_uint32, c_uint64, c_uint32, c_void_p, c_size_t, POINTER(c_size_t), c_int],
    ),
    "kman_format_uniq": (
        c_int,
        [c_void_p, c_void_p, c_uint32, c_uint64, c_uint32, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p,
         c_size_t, POINTER(c_size_t), c_int],
    ),
}

_lib = None
_lock = threading.Lock()


def header_symbols() -> list:
    """Function names declared in include/kman.h (parsed, for the ABI test)."""
    import re

    path = os.path.join(os.path.dirname(HERE), "include", "kman.h")
    with open(path) as fh:
        text = fh.read()
    return sorted(set(re.findall(r"\b(kman_[a-z0-9_]+)\s*\(", text)))


def lib() -> ctypes.CDLL:
    """Load libkman.so once; raise loudly if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.isfile(LIB_PATH):
                raise RuntimeError(
                    "libkman.so not found at %s: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                    "(the MI355X engine has no CPU fallback)" % LIB_PATH
                )
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def check(ctx, rc: int, what: str) -> None:
    if rc == KMAN_OK:
        return
    msg = lib().kman_last_error(ctx).decode(errors="replace") if ctx else ""
    if rc in (KMAN_EINVAL, KMAN_EFORMAT):
        raise AssertionError(msg or what)
    if rc == KMAN_ENOMEM:
        raise MemoryError("%s: %s" % (what, msg))
    raise RuntimeError("%s failed (%d): %s" % (what, rc, msg))


def device_count() -> int:
    n = c_int(0)
    lib().kman_device_count(ctypes.byref(n))
    return n.value
