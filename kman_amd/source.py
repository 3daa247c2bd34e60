"""Device-resident k-mer sources behind the Batch objects.

A ``FastaSource`` is one parsed FASTA input on one GPU (one
``FastaBatcher.do`` call): the cleaned base codes and the record table stay in
HBM, k-mer keys (+ pos payloads) are extracted on demand in the reference's
stream order.  A ``Batch`` of the reference is a view ``[start, end)`` of that
stream (BatcherBase.new_batch/add_record, batcher.py:118-131).

A ``BatchFileSource`` is a folder of batch FASTA files written by
``kmer batch`` (records ``>ref:start-end:strand`` / k-mer), loaded back for
``-B``: every record is one k-mer whose header is its title.
"""

from __future__ import annotations

import ctypes
import os
from ctypes import byref, c_int, c_void_p
from typing import List, Optional

import numpy as np

from . import _native as N
from . import engine, phases


class FastaSource:
    def __init__(self, dev: engine.Device, text: Optional[bytes], k: int, rc: bool, path: Optional[str] = None):
        """The k-mer stream of FASTA bytes (`text`), or of the file at `path`
        (engine.parse_file: chunked pinned reads overlapping the H2D)."""
        engine._check_k(k, wide=True)
        self.dev, self.k, self.rc = dev, k, rc
        self.parsed = engine.parse_file(dev, path) if text is None else engine.parse(dev, text)
        engine.check_empty_names(self.parsed, k)
        self.n_kmers = engine.count_kmers(self.parsed, k, rc)
        self._km = {}  # want_pos -> engine.Kmers (stream order)
        phases.mark("count_kmers")

    # ------------------------------------------------------------ extraction
    def kmers(self, want_pos: bool):
        """Keys (+ pos) in stream order -- engine.Kmers (u64 keys, k <= 32)
        or engine.Words (word planes, k > 32); the cached arrays are never
        sorted in place (sorts work on copies)."""
        km = self._km.get(want_pos) or (self._km.get(True) if not want_pos else None)
        if km is None:
            if self.k > engine.MAX_K:
                km = engine.extract_words(self.parsed, self.k, self.rc, want_pos=True)
                self._km[True] = km
                return km
            km = engine.extract(self.parsed, self.k, self.rc, want_pos=want_pos)
            self._km[want_pos] = km
        return km

    def header(self, pos: int) -> str:
        p = int(pos) >> 1
        r = self.parsed.record_of(p)
        st = p - int(self.parsed.rec_seq[r])
        name = self.parsed.names[r].decode("utf-8", "surrogateescape")
        return "%s:%d-%d:%s" % (name, st, st + self.k, "-" if int(pos) & 1 else "+")

    def format_fasta(self, keys: np.ndarray, pos: np.ndarray) -> bytes:
        if keys.ndim == 2:  # word keys (k > 32): (n, W)
            return engine.format_fasta_words(keys, pos, self.k, self.parsed)
        return engine.format_fasta(keys, pos, self.k, self.parsed)

    def free(self) -> None:
        for km in self._km.values():
            km.free()
        self._km.clear()
        self.parsed.free()


class BatchFileSource:
    """Batch FASTA files (``kmer batch`` output) loaded back onto the GPU."""

    def __init__(self, dev: engine.Device, paths: List[str]):
        self.dev = dev
        self.paths = list(paths)
        texts = [engine.read_input(p) for p in self.paths]
        self.file_of_record: List[int] = []
        blob = []
        for i, t in enumerate(texts):
            if t and not t.endswith(b"\n"):
                t += b"\n"
            blob.append(t)
        text = b"".join(blob)
        self.k = 0
        self.n_kmers = 0
        self._km = None
        if not text.strip():
            self.parsed = None
            self.titles: List[str] = []
            self.file_sizes = [0] * len(paths)
            return
        self.parsed = engine.parse(dev, text)
        lens = np.diff(np.append(self.parsed.rec_seq, np.uint64(self.parsed.n_bases))).astype(np.int64)
        if len(lens) and (lens != lens[0]).any():
            raise AssertionError("batch files mix k-mer lengths")
        self.k = int(lens[0]) if len(lens) else 0
        self.titles = [self._title(text, int(h)) for h in self.parsed.rec_hdr]
        self.n_kmers = engine.count_kmers(self.parsed, self.k, False) if self.k > 1 else 0
        # records per file, for Batch sizes
        ends = np.cumsum([len(b) for b in blob])
        self.file_sizes = list(np.bincount(np.searchsorted(ends, self.parsed.rec_hdr, side="right"),
                                           minlength=len(paths)))

    @staticmethod
    def _title(text: bytes, h: int) -> str:
        j = h + 1
        while j < len(text) and text[j] not in (10, 13):
            j += 1
        return text[h + 1 : j].decode("utf-8", "surrogateescape").rstrip()

    def kmers(self, want_pos: bool):
        if self._km is None:
            if self.k > engine.MAX_K:
                self._km = engine.extract_words(self.parsed, self.k, False, want_pos=True)
            else:
                self._km = engine.extract(self.parsed, self.k, False, want_pos=True)
        return self._km

    def header(self, pos: int) -> str:
        return self.titles[self.parsed.record_of(int(pos) >> 1)]

    def format_fasta(self, keys: np.ndarray, pos: np.ndarray) -> bytes:
        from .join import format_sources

        return format_sources(keys, pos, self.k, [self], False)

    def free(self) -> None:
        if self._km is not None:
            self._km.free()
        if self.parsed is not None:
            self.parsed.free()


# ------------------------------------------------------------------ sorting


def sorted_copy(src, start: int, end: int, want_pos: bool, per_batch: Optional[int] = None):
    """Stable sort of stream range [start, end) of a source (device copy).

    With ``per_batch`` the range is cut into consecutive chunks of that many
    k-mers, counted from stream index 0, and every chunk is sorted on its own
    (the reference sorts each Batch separately, batch.py:156-168)."""
    dev = src.dev
    km = src.kmers(want_pos)
    n = end - start
    L = N.lib()
    if isinstance(km, engine.Words):
        # word keys (k > 32): an LSD sort over the planes of the range (a
        # view of the cached planes: same stride, offset by start)
        view = engine.Words(_Ptr(km.words.ptr + 8 * start, dev), _Ptr(km.pos.ptr + 8 * start, dev)
                            if (want_pos and km.pos is not None) else None, n, src.k, km.stride)
        return engine.sort_words(view, start=start, per_batch=per_batch, dev=dev)
    out = engine.Kmers(dev.alloc(8 * max(n, 1)), dev.alloc(8 * max(n, 1)), None, None, 0, n, src.k,
                       dev.alloc(8 * 256 * 8))
    N.check(dev.ctx, L.kman_memcpy_d2d(dev.ctx, c_void_p(out.keys.ptr), c_void_p(km.keys.ptr + 8 * start), 8 * n),
            "d2d")
    if want_pos:
        pb = km.pos_bytes
        out.pos, out.pos_alt, out.pos_bytes = dev.alloc(pb * max(n, 1)), dev.alloc(pb * max(n, 1)), pb
        N.check(dev.ctx, L.kman_memcpy_d2d(dev.ctx, c_void_p(out.pos.ptr), c_void_p(km.pos.ptr + pb * start),
                                            pb * n), "d2d")
    key_bits = 2 * src.k
    if per_batch is not None and n:
        nb_last = (start + n - 1) // per_batch
        tag_bits = max(1, int(nb_last).bit_length())
        if key_bits + tag_bits <= 64:
            N.check(dev.ctx, L.kman_tag_batches(dev.ctx, c_void_p(out.keys.ptr), n, key_bits, start, per_batch),
                    "tag")
            _sort(out, dev, key_bits + tag_bits)
            return out
        # no room for a tag: sort each chunk on its own
        b = start
        while b < end:
            e = min(end, (b // per_batch + 1) * per_batch)
            sub = engine.Kmers(_Ptr(out.keys.ptr + 8 * (b - start)), _Ptr(out.alt.ptr + 8 * (b - start)),
                               _Ptr(out.pos.ptr + out.pos_bytes * (b - start)) if out.pos else None,
                               _Ptr(out.pos_alt.ptr + out.pos_bytes * (b - start)) if out.pos else None,
                               out.pos_bytes, e - b, src.k, out.hist)
            flipped = _sort(sub, dev, key_bits, copy_back=True)
            assert not flipped
            b = e
        return out
    _sort(out, dev, key_bits)
    return out


class _Ptr:
    """A raw device pointer viewed like a DeviceBuffer (no ownership)."""

    def __init__(self, ptr, dev=None):
        self.ptr = ptr
        self.dev = dev

    def free(self):
        pass


def _sort(km: engine.Kmers, dev: engine.Device, key_bits: int, copy_back: bool = False) -> bool:
    res = c_int(0)
    L = N.lib()
    rc = L.kman_sort(dev.ctx, c_void_p(km.keys.ptr), c_void_p(km.alt.ptr), c_void_p(km.pos.ptr if km.pos else None),
                     c_void_p(km.pos_alt.ptr if km.pos_alt else None), km.pos_bytes, km.n, key_bits, None,
                     byref(res))
    N.check(dev.ctx, rc, "kman_sort")
    if res.value:
        if copy_back:
            L.kman_memcpy_d2d(dev.ctx, c_void_p(km.keys.ptr), c_void_p(km.alt.ptr), 8 * km.n)
            if km.pos is not None:
                L.kman_memcpy_d2d(dev.ctx, c_void_p(km.pos.ptr), c_void_p(km.pos_alt.ptr), km.pos_bytes * km.n)
            return False
        km.keys, km.alt = km.alt, km.keys
        km.pos, km.pos_alt = km.pos_alt, km.pos
    km.sorted = True
    return bool(res.value) and not copy_back


def download_sorted(src, start: int, end: int, want_pos: bool, per_batch: Optional[int] = None):
    """Sorted keys (u64, or (n, W) word rows for k > 32) and pos on the host."""
    km = sorted_copy(src, start, end, want_pos, per_batch)
    if isinstance(km, engine.Words):
        try:
            keys = engine.download_words(src.dev, km.words, km.n, src.k, km.stride)
            pos = src.dev.download(km.pos, km.n, np.uint64) if want_pos else None
        finally:
            km.free()
        return keys, pos
    try:
        mask = np.uint64((1 << (2 * src.k)) - 1) if src.k < 32 else np.uint64(0xFFFFFFFFFFFFFFFF)
        keys = src.dev.download(km.keys, km.n, np.uint64) & mask
        pos = None
        if want_pos:
            pos = src.dev.download(km.pos, km.n, np.uint32 if km.pos_bytes == 4 else np.uint64)
    finally:
        km.free()
    return keys, pos


# ------------------------------------------------------------- gather + sort


def gather_sorted(entries, want_pos: bool):
    """Concatenate stream ranges ``(src, start, end)`` (in batch order) into
    one device array and sort it stably: the device form of the reference's
    heap n-way merge of sorted batches (join.py:63-93; ties by batch order,
    then in-batch order).  With several sources the pos payload becomes u64
    tagged with the source index in bits 56-63.

    Returns (engine.Kmers sorted on device, list of sources, tagged)."""
    srcs = []
    for s, _, _ in entries:
        if not any(s is x for x in srcs):
            srcs.append(s)
    ks = {s.k for s in srcs}
    if len(ks) != 1:
        raise AssertionError("batches of different k cannot be joined")
    k = ks.pop()
    tagged = len(srcs) > 1
    if tagged and len(srcs) > 255:
        raise AssertionError("at most 255 sources per join")
    dev = srcs[0].dev
    L = N.lib()
    n = sum(e - s for _, s, e in entries)
    if k > engine.MAX_K:
        return _gather_sorted_words(entries, srcs, tagged, k, n, want_pos), srcs, tagged
    pb = 8 if tagged else (srcs[0].kmers(want_pos).pos_bytes if want_pos else 0)
    out = engine.Kmers(dev.alloc(8 * max(n, 1)), dev.alloc(8 * max(n, 1)), None, None, 0, n, k,
                       dev.alloc(8 * 256 * 8))
    if want_pos:
        out.pos, out.pos_alt, out.pos_bytes = dev.alloc(pb * max(n, 1)), dev.alloc(pb * max(n, 1)), pb
    at = 0
    for src, s, e in entries:
        m = e - s
        if m <= 0:
            continue
        km = src.kmers(want_pos)
        N.check(dev.ctx, L.kman_memcpy_d2d(dev.ctx, c_void_p(out.keys.ptr + 8 * at), c_void_p(km.keys.ptr + 8 * s),
                                            8 * m), "d2d")
        if want_pos:
            tag = next(i for i, x in enumerate(srcs) if x is src) << 56 if tagged else 0
            if km.pos_bytes == pb:
                N.check(dev.ctx, L.kman_memcpy_d2d(dev.ctx, c_void_p(out.pos.ptr + pb * at),
                                                    c_void_p(km.pos.ptr + pb * s), pb * m), "d2d")
                if tag:
                    N.check(dev.ctx, L.kman_or_u64(dev.ctx, c_void_p(out.pos.ptr + 8 * at), m, tag), "tag")
            else:  # u32 source payload into the u64 tagged array
                N.check(dev.ctx, L.kman_widen_u32(dev.ctx, c_void_p(km.pos.ptr + 4 * s),
                                                   c_void_p(out.pos.ptr + 8 * at), m, tag), "widen")
        at += m
    if all(isinstance(s, BatchFileSource) for s, _, _ in entries) and _merge_sorted_runs(out, entries, dev):
        return out, srcs, tagged
    _sort(out, dev, 2 * k)
    return out, srcs, tagged


def _merge_sorted_runs(out: engine.Kmers, entries, dev: engine.Device) -> bool:
    """Batch files written by `kmer batch` are each sorted: their union is
    merged (kman_merge_runs, the device form of Crawler.do_records'
    heapq.merge, join.py:63-93) instead of sorted; equal keys keep batch
    order, then in-batch order, as the heap merge does.  False (nothing
    changed) when a run is not sorted after all -- the caller sorts."""
    L = N.lib()
    runs, at = [], 0
    for _, s, e in entries:
        m = e - s
        if m <= 0:
            continue
        d = ctypes.c_uint64(0)
        N.check(dev.ctx, L.kman_count_descents(dev.ctx, c_void_p(out.keys.ptr + 8 * at), m, byref(d)), "descents")
        if d.value:
            return False
        runs.append(N.Run(out.keys.ptr + 8 * at, out.pos.ptr + out.pos_bytes * at if out.pos else None, m))
        at += m
    if len(runs) < 2:
        out.sorted = True
        return True
    pb = out.pos_bytes if out.pos else 0
    tk = dev.alloc(8 * max(at, 1))
    tv = dev.alloc(pb * max(at, 1)) if pb else None
    try:
        arr = (N.Run * len(runs))(*runs)
        N.check(dev.ctx, L.kman_merge_runs(dev.ctx, arr, len(runs), pb, c_void_p(out.alt.ptr),
                                           c_void_p(out.pos_alt.ptr) if pb else None, c_void_p(tk.ptr),
                                           c_void_p(tv.ptr) if tv else None), "kman_merge_runs")
    finally:
        tk.free()
        if tv is not None:
            tv.free()
    out.keys, out.alt = out.alt, out.keys
    out.pos, out.pos_alt = out.pos_alt, out.pos
    out.sorted = True
    return True


def _gather_sorted_words(entries, srcs, tagged: bool, k: int, n: int, want_pos: bool) -> engine.Words:
    """gather_sorted for word keys (k > 32): the ranges' planes concatenated
    in batch order (pos tagged with the source index in bits 56-63 when
    several sources are joined), then one stable LSD sort over the planes --
    the heap merge's order (ties by batch, then in-batch order)."""
    dev = srcs[0].dev
    L = N.lib()
    W = engine.nwords(k)
    cat = engine.Words(dev.alloc(8 * W * max(n, 1)), dev.alloc(8 * max(n, 1)) if want_pos else None, n, k,
                       max(n, 1))
    try:
        at = 0
        for src, s, e in entries:
            m = e - s
            if m <= 0:
                continue
            km = src.kmers(True)
            for j in range(W):
                N.check(dev.ctx, L.kman_memcpy_d2d(dev.ctx, c_void_p(cat.plane(j) + 8 * at),
                                                    c_void_p(km.plane(j) + 8 * s), 8 * m), "d2d")
            if want_pos:
                N.check(dev.ctx, L.kman_memcpy_d2d(dev.ctx, c_void_p(cat.pos.ptr + 8 * at),
                                                    c_void_p(km.pos.ptr + 8 * s), 8 * m), "d2d")
                if tagged:
                    tag = next(i for i, x in enumerate(srcs) if x is src) << 56
                    if tag:
                        N.check(dev.ctx, L.kman_or_u64(dev.ctx, c_void_p(cat.pos.ptr + 8 * at), m, tag), "tag")
            at += m
        return engine.sort_words(cat, dev=dev)
    finally:
        cat.free()
