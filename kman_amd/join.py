"""K-way join of k-mer batches (kmermaid/join.py).

``KJoiner.join(batches, outpath)`` is the reference's n-way heap merge +
run-length grouping + count/uniq writer (join.py:63-130, 244-285, 376-391).
On the GPU the n-way merge of sorted batches is one stable radix sort of the
union of the batches' k-mers (its result is exactly the merged order — ties
in batch, then in-batch order, i.e. stream order) followed by the RLE kernel:

* SEQ_COUNT -> kman_rle_count  -> ``"%s\\t%d\\n"``
* UNIQUE    -> kman_rle_uniq   -> ``">%s\\n%s\\n"`` (groups of exactly one)

Outputs do not depend on how the stream was cut into batches (verified on
the reference), so batches that come from one FastaBatcher run
are joined as the whole device-resident stream without materialising them.

VEC_COUNT / VEC_COUNT_MASKED (join.py:288-335): the reference's
AbundanceVector.add_count first calls its abstract base (abundance.py:60,123),
which raises NotImplementedError, so its join stops at the first add_count:
VEC_COUNT at the first k-mer, VEC_COUNT_MASKED at the first k-mer seen in two
records of different names (join.py:318-335); a join that never calls it
writes the empty vector folder (abundance.py:151-172).  That is the default
here too (the device answers whether add_count would be called).  With
``KMAN_VEC_COUNT=1`` they instead do what the code around that call evidently
means (abundance.py:103-168): one vector per (record, strand) indexed by
window start, holding the k-mer's count (VEC_COUNT) or its occurrences in
other records when it occurs in more than one (VEC_COUNT_MASKED), written as
``<out>/<ref>___<strand>.gz`` = "# k=<k>" + one count per line.  The counts
come from one device sort + kman_vec_fill; tests/test_gpu_vectors.py checks
them against a restatement of that code (parity unpinned: the reference
never produces a vector).
"""

from __future__ import annotations

import gzip
import logging
import os
import tempfile
from enum import Enum
from typing import Dict, Iterator, List, Tuple

import numpy as np

from . import engine, phases
from .batch import Batch


def _entries(batches: List[Batch]):
    """(source, start, end) of every non-empty device batch, in batch order."""
    out = []
    for b in batches:
        if b is None or b.current_size == 0:
            continue
        if not b.on_device:
            raise AssertionError("host-mode batches are not k-mer batches")
        s, e = b.stream_range
        out.append((b.source, s, e))
    return out


def _whole_stream(entries):
    """The FastaSource whose whole k-mer stream the entries cover exactly once
    (any batch order), else None."""
    from .source import FastaSource

    src = entries[0][0]
    if not isinstance(src, FastaSource) or any(s is not src for s, _, _ in entries):
        return None
    at = 0
    for _, s, e in sorted(entries, key=lambda x: x[1]):
        if s != at:
            return None
        at = e
    return src if at == src.n_kmers else None


class Crawler:
    """Merged crawl over batches (join.py:36-130)."""

    doSort = False
    doSmart = False
    verbose = True
    desc = ""

    @staticmethod
    def count_records(batches: List[Batch]) -> int:
        return sum(b.current_size for b in batches)

    def do_records(self, batches: List[Batch]) -> Iterator[Tuple[str, str]]:
        """(header, seq) of every record in merged order (heap-merge order),
        from one stable device sort of the union of the batches."""
        if any(type(b) is not Batch for b in batches):
            raise AssertionError()
        entries = _entries(batches)
        if not entries:
            return
        from .source import gather_sorted

        km, srcs, tagged = gather_sorted(entries, want_pos=True)
        k = srcs[0].k
        try:
            dev = srcs[0].dev
            if isinstance(km, engine.Words):  # (k > 32: word rows)
                keys = engine.download_words(dev, km.words, km.n, k, km.stride)
                pos = dev.download(km.pos, km.n, np.uint64)
                dec = lambda x: engine.decode_words(x, k)  # noqa: E731
            else:
                keys = dev.download(km.keys, km.n, np.uint64)
                pos = dev.download(km.pos, km.n, np.uint32 if km.pos_bytes == 4 else np.uint64)
                dec = lambda x: engine.decode_key(x, k)  # noqa: E731
        finally:
            km.free()
        for key, p in zip(keys.tolist(), pos.tolist()):
            src = srcs[p >> 56] if tagged else srcs[0]
            yield (src.header(p & ((1 << 56) - 1)), dec(key))

    def do_batch(self, batches: List[Batch]) -> Iterator[Tuple[List[str], str]]:
        crawler = self.do_records(batches)
        try:
            first = next(crawler)
        except StopIteration:
            logging.error("nothing to crawl")
            return
        cur_seq, cur_headers = first[1], [first[0]]
        for header, seq in crawler:
            if seq == cur_seq:
                cur_headers.append(header)
            else:
                yield (cur_headers, cur_seq)
                cur_seq, cur_headers = seq, [header]
        yield (cur_headers, cur_seq)


class KJoiner:
    class MODE(Enum):
        UNIQUE = 1
        SEQ_COUNT = 2
        VEC_COUNT = 3
        VEC_COUNT_MASKED = 4

    class MEMORY(Enum):
        NORMAL = 1
        LOCAL = 2

    DEFAULT_MODE = MODE.UNIQUE
    DEFAULT_MEMORY = MEMORY.NORMAL

    def __init__(self, mode: "KJoiner.MODE" = None, memory: "KJoiner.MEMORY" = None):
        self.__mode = self.DEFAULT_MODE
        self.__memory = self.DEFAULT_MEMORY
        if mode is not None:
            if not isinstance(mode, self.MODE):
                raise AssertionError
            self.__mode = mode
        if memory is not None:
            if not isinstance(memory, self.MEMORY):
                raise AssertionError
            self.__memory = memory

    @property
    def mode(self):
        return self.__mode

    @mode.setter
    def mode(self, mode) -> None:
        if not isinstance(mode, self.MODE):
            raise AssertionError
        self.__mode = mode

    @property
    def memory(self):
        return self.__memory

    @memory.setter
    def memory(self, memory) -> None:
        if not isinstance(memory, self.MEMORY):
            raise AssertionError
        self.__memory = memory

    @staticmethod
    def join_unique(headers: List[str], seq: str, OH, **kwargs):
        if len(headers) != 1:
            return None
        OH.write(">%s\n%s\n" % (headers[0], seq))
        return (headers[0], seq)

    @staticmethod
    def join_sequence_count(headers: List[str], seq: str, OH, **kwargs):
        OH.write("%s\t%d\n" % (seq, len(headers)))
        return (seq, len(headers))

    @property
    def join_function(self):
        return {self.MODE.UNIQUE: self.join_unique, self.MODE.SEQ_COUNT: self.join_sequence_count}.get(self.mode)

    def join(self, batches: List[Batch], outpath: str) -> None:
        """Join batches into ``outpath`` on the GPU (join.py:376-391)."""
        print("Joining...")
        from .launch import ShardedSource

        sharded = [b for b in batches if b is not None and isinstance(b.source, ShardedSource)]
        if sharded:
            # one rank of a multi-GPU run (kman_amd/launch.py): the key rounds
            # across the ranks, every rank writing its slice of `outpath`
            others = [b for b in batches if b is not None and b.current_size and b not in sharded]
            if self.mode.name.startswith("VEC_") or others or len(sharded) != 1:
                raise NotImplementedError("a multi-GPU launch joins the FastaBatcher shard batches by UNIQUE / "
                                          "SEQ_COUNT only")
            sharded[0].source.join(self.mode == self.MODE.SEQ_COUNT, outpath)
            return
        if self.mode.name.startswith("VEC_"):
            join_vectors(batches, self.mode == self.MODE.VEC_COUNT_MASKED, outpath)
            return
        with open(outpath, "wb") as OH:
            join_bytes(batches, self.mode == self.MODE.SEQ_COUNT, sink=OH)


def join_bytes(batches: List[Batch], count: bool, sink=None):
    """Device join of the batches: gather + stable sort + RLE, then format.
    Returns the output text, or writes it to the binary file `sink`."""
    entries = _entries(batches)
    if not entries:
        logging.error("nothing to crawl")  # join.py:110; the output stays empty
        return None if sink is not None else b""
    from .source import gather_sorted

    whole = _whole_stream(entries)
    if whole is not None:
        # the batches are one FASTA stream, each k-mer once: count / uniq do
        # not depend on the batch cut, so the stream goes
        # straight from the codes: region path, else the multi-batch join when
        # one batch does not fit the HBM, else the general path (no copy of a
        # cached extraction either way)
        r = engine.join_groups(whole.parsed, whole.k, whole.rc, "count" if count else "uniq")
        phases.mark("step")
        if r is None:
            return None if sink is not None else b""
        try:
            if isinstance(r, engine.WordsResult):
                return engine._emit_words(whole.parsed, r, sink)
            if count:
                return engine.emit_count(whole.dev, r, sink)
            return engine.emit_uniq(whole.parsed, r, sink)
        finally:
            phases.mark("format+d2h+write")
            engine.free_result(r)
    km, srcs, tagged = gather_sorted(entries, want_pos=not count)
    dev = srcs[0].dev
    k = srcs[0].k
    if isinstance(km, engine.Words):  # word keys (k > 32): several sources, or reloaded batch files
        try:
            r = engine.rle_words(km, "count" if count else "uniq")
        finally:
            km.free()
        try:
            if count:
                return engine._emit_words(_any_parsed(srcs), r, sink)
            rows = engine.download_words(dev, r.words, r.n, k, max(r.n, 1))
            pos = dev.download(r.vals, r.n, np.uint64)
        finally:
            r.free()
        return engine._to(sink, format_sources(rows, pos, k, srcs, tagged))
    try:
        if count:
            r = engine.rle_count(km, dev)
            try:
                return engine.emit_count(dev, r, sink)
            finally:
                r.ukeys.free()
                r.counts.free()
        r = engine.rle_uniq(km, dev)
        try:
            keys, pos = engine.download_uniq(dev, r)
        finally:
            r.keys.free()
            r.pos.free()
    finally:
        km.free()
    return engine._to(sink, format_sources(keys, pos, k, srcs, tagged))


def vectors_enabled() -> bool:
    """KMAN_VEC_COUNT=1: write abundance vectors (this engine's semantics);
    otherwise VEC_* behave as the reference (NotImplementedError at its first
    add_count)."""
    return os.environ.get("KMAN_VEC_COUNT") == "1"


def _any_parsed(srcs):
    """A parsed source (only its device is used by the count writers)."""
    for s in srcs:
        if getattr(s, "parsed", None) is not None:
            return s.parsed
    raise AssertionError("no parsed source")


def join_vectors(batches: List[Batch], masked: bool, outpath: str) -> None:
    """Abundance vectors of the joined batches (module docstring): the union
    sorted on the device (gather_sorted), each item's count (or masked count)
    written at its (source, window, strand) slot by kman_vec_fill, then one
    gzip file per (record, strand) that received a count, its vector running
    to the last such window (AbundanceVector.add_ref grows it to pos + 1).
    Without KMAN_VEC_COUNT=1: NotImplementedError wherever the reference's
    add_count would be called, else the empty folder."""
    emulate = not vectors_enabled()
    import ctypes
    from ctypes import byref, c_size_t, c_void_p

    from . import _native as N
    from .source import FastaSource, gather_sorted

    dirpath = os.path.splitext(outpath)[0]
    entries = _entries(batches)
    if not entries:
        logging.error("nothing to crawl")  # join.py:110; then write_to with no vectors
        if os.path.isfile(dirpath):
            raise AssertionError
        print('Writing output in "%s"' % dirpath)
        os.makedirs(dirpath, exist_ok=True)
        return
    if os.path.isfile(dirpath):
        raise AssertionError
    if emulate and not masked:
        # (the first group's add_count raises, abundance.py:60 via :123)
        raise NotImplementedError("AbundanceVector.add_count (the reference's VEC_COUNT)")
    if emulate and (not all(isinstance(e[0], FastaSource) for e in entries) or entries[0][0].k > engine.MAX_K):
        # reloaded batch files (-B) or word keys (k > 32): the same decision
        # from the sorted union on the host side (bounded slices)
        if groups_span_refs(entries):
            raise NotImplementedError("AbundanceVector.add_count (the reference's VEC_COUNT_MASKED)")
        print('Writing output in "%s"' % dirpath)  # abundance.py:160: no vector was added
        os.makedirs(dirpath, exist_ok=True)
        return
    if not all(isinstance(e[0], FastaSource) for e in entries):
        raise NotImplementedError("abundance vectors of reloaded batch files (-B)")
    if entries[0][0].k > engine.MAX_K:
        raise NotImplementedError("abundance vectors of k > 32 (word keys)")
    km, srcs, tagged = gather_sorted(entries, want_pos=True)
    dev, k, L = srcs[0].dev, srcs[0].k, N.lib()
    base = np.concatenate([[0], np.cumsum([2 * s.parsed.n_bases for s in srcs])]).astype(np.uint64)
    total = int(base[-1])
    # record identity = record name (SequenceCoords.from_str: ref); two
    # records of one name would share a vector and collide in add_count
    names, rec_start, rec_end = [], [], []
    for si, s in enumerate(srcs):
        p = s.parsed
        rs = np.asarray(p.rec_seq, dtype=np.uint64)
        ends = np.append(rs[1:], np.uint64(p.n_bases))
        names += list(p.names)
        rec_start.append(base[si] + 2 * rs)
        rec_end.append(base[si] + 2 * ends)
    if emulate:
        # masked counts by record NAME (the reference's ref): nonzero exactly
        # where a group holds two refs, i.e. where add_count would be called
        rec_id = np.unique(np.asarray(names, dtype=object), return_inverse=True)[1].astype(np.uint32)
    elif len(set(names)) != len(names):
        raise AssertionError("abundance vectors need distinct record names (one vector per ref:strand)")
    else:
        rec_id = np.arange(len(names), dtype=np.uint32)
    rec_start = np.concatenate(rec_start).astype(np.uint64)
    rec_end = np.concatenate(rec_end).astype(np.uint64)
    bufs = []
    vec = None
    try:
        vec = dev.alloc(4 * max(total, 1))
        dev.memset(vec, 0, 4 * max(total, 1))
        d_base, d_rs, d_id = dev.alloc(8 * len(base)), dev.alloc(8 * max(1, len(rec_start))), dev.alloc(
            4 * max(1, len(rec_id)))
        bufs += [d_base, d_rs, d_id]
        dev.upload(d_base, base)
        dev.upload(d_rs, rec_start)
        dev.upload(d_id, rec_id)
        N.check(dev.ctx, L.kman_vec_fill(dev.ctx, c_void_p(km.keys.ptr), c_void_p(km.pos.ptr), km.pos_bytes, km.n,
                                         1 if masked else 0, c_void_p(d_base.ptr), 1 if tagged else 0,
                                         c_void_p(d_rs.ptr), c_void_p(d_id.ptr), len(rec_start), c_void_p(vec.ptr)),
                "kman_vec_fill")
        km.free()
        km = None
        for b in bufs:
            b.free()
        bufs = []
        # the slots stay in HBM (8 B per base): the host takes bounded slices
        if emulate:
            for lo in range(0, total, _VEC_SLICE):
                if dev.download(vec, min(_VEC_SLICE, total - lo), np.uint32, 4 * lo).any():
                    raise NotImplementedError("AbundanceVector.add_count (the reference's VEC_COUNT_MASKED)")
            print('Writing output in "%s"' % dirpath)  # abundance.py:160: no vector was added
            os.makedirs(dirpath, exist_ok=True)
            return
        print('Writing output in "%s"' % dirpath)  # abundance.py:160
        os.makedirs(dirpath, exist_ok=True)
        for r, name in enumerate(names):
            for strand in (0, 1):
                n = _vector_len(dev, vec, int(rec_start[r]) + strand, int(rec_end[r]))
                if not n:
                    continue  # no add_count for this ref:strand: no vector, no file
                arr = np.empty(n, np.uint32)
                for lo in range(0, n, _VEC_SLICE // 2):
                    m = min(_VEC_SLICE // 2, n - lo)
                    arr[lo:lo + m] = dev.download(vec, 2 * m - 1, np.uint32,
                                                  4 * (int(rec_start[r]) + strand + 2 * lo))[::2]
                used = c_size_t(0)
                rc = L.kman_format_vector(arr.ctypes.data_as(c_void_p), n, 1, None, 0, byref(used),
                                          engine.host_threads())
                if rc not in (N.KMAN_OK, N.KMAN_ECAP):
                    raise RuntimeError("kman_format_vector failed (%d)" % rc)
                buf = ctypes.create_string_buffer(max(1, used.value))
                rc = L.kman_format_vector(arr.ctypes.data_as(c_void_p), n, 1, buf, used.value, byref(used),
                                          engine.host_threads())
                if rc != N.KMAN_OK:
                    raise RuntimeError("kman_format_vector failed (%d)" % rc)
                ref = name.decode("utf-8", "surrogateescape")
                with gzip.open(os.path.join(dirpath, "%s___%s.gz" % (ref, "+-"[strand])), "wb") as OH:
                    OH.write(b"# k=%d\n" % k)
                    OH.write(buf.raw[:used.value])
    finally:
        if km is not None:
            km.free()
        for b in bufs:
            b.free()
        if vec is not None:
            vec.free()


_VEC_SLICE = 1 << 26  # u32 slots per host slice (256 MiB)
_GROUP_SLICE = 1 << 24  # items per host slice of groups_span_refs


def _record_refs(src, ref_ids: dict) -> Tuple[np.ndarray, np.ndarray]:
    """(first base of each record, ref id of each record) of one source.
    The ref is what SequenceCoords.from_str reads from the record's header
    (join.py:311-335): a FASTA record's name, or the ref field of a batch
    file record's title (seq.py:106-127; an incompatible title raises
    AssertionError, as the reference does at that group)."""
    from .seq import SequenceCoords
    from .source import FastaSource

    if isinstance(src, FastaSource):
        names = [n.decode("utf-8", "surrogateescape") for n in src.parsed.names]
    else:
        names = [SequenceCoords.from_str(t).ref for t in src.titles]
    ids = np.array([ref_ids.setdefault(nm, len(ref_ids)) for nm in names], np.int64)
    return np.asarray(src.parsed.rec_seq, np.uint64), ids


def groups_span_refs(entries) -> bool:
    """True iff some group of equal k-mers of the joined batches holds
    records of two different refs: exactly when the reference's
    join_vector_count_masked reaches AbundanceVector.add_count
    (join.py:318-335, which raises NotImplementedError, abundance.py:60 via
    :123).  The union is sorted on the device (gather_sorted: any k, FASTA
    or batch-file sources); groups and their min / max ref are found on the
    host in bounded slices, a group open at a slice end carried over."""
    from .source import gather_sorted

    km, srcs, tagged = gather_sorted(entries, want_pos=True)
    try:
        dev, k = srcs[0].dev, srcs[0].k
        ref_ids: dict = {}
        recs = [_record_refs(s, ref_ids) for s in srcs]
        if len(ref_ids) < 2:
            return False
        words = isinstance(km, engine.Words)
        W = engine.nwords(k) if words else 1
        pb = 8 if words else km.pos_bytes
        mask = np.uint64((1 << (2 * k)) - 1) if k < 32 else np.uint64(0xFFFFFFFFFFFFFFFF)
        low56 = np.uint64((1 << 56) - 1)
        carry = None  # (key row, min ref, max ref) of the group open at the last slice's end
        for lo in range(0, km.n, _GROUP_SLICE):
            m = min(_GROUP_SLICE, km.n - lo)
            if words:
                keys = np.stack([dev.download(_Raw(km.plane(j)), m, np.uint64, 8 * lo) for j in range(W)], axis=1)
            else:
                keys = (dev.download(km.keys, m, np.uint64, 8 * lo) & mask)[:, None]
            pos = dev.download(km.pos, m, np.uint64 if pb == 8 else np.uint32, pb * lo).astype(np.uint64)
            base = (pos & low56) >> np.uint64(1)
            src_of = (pos >> np.uint64(56)).astype(np.int64) if tagged else np.zeros(m, np.int64)
            ref = np.empty(m, np.int64)
            for si, (rs, ids) in enumerate(recs):
                sel = src_of == si
                if sel.any():
                    ref[sel] = ids[np.searchsorted(rs, base[sel], side="right") - 1]
            new = np.ones(m, bool)
            new[1:] = (keys[1:] != keys[:-1]).any(axis=1)
            if carry is not None and (keys[0] == carry[0]).all():
                new[0] = False
            starts = np.flatnonzero(new)
            if not new[0]:  # the carried group continues into this slice
                end0 = int(starts[0]) if len(starts) else m
                carry = (carry[0], min(carry[1], int(ref[:end0].min())), max(carry[2], int(ref[:end0].max())))
            if len(starts):
                if carry is not None and carry[1] != carry[2]:
                    return True
                mins = np.minimum.reduceat(ref, starts)
                maxs = np.maximum.reduceat(ref, starts)
                if (mins[:-1] != maxs[:-1]).any():
                    return True
                carry = (keys[-1].copy(), int(mins[-1]), int(maxs[-1]))
        return carry is not None and carry[1] != carry[2]
    finally:
        km.free()


class _Raw:
    """A raw device pointer for Device.download (no ownership)."""

    def __init__(self, ptr: int):
        self.ptr = ptr


def _vector_len(dev, vec, first: int, end: int) -> int:
    """Length of one (record, strand) vector: its last nonzero slot + 1
    (slots first, first + 2, .. < end), found from the back in bounded
    slices; 0 when the record's strand received no count."""
    n_slots = (end - first + 1) // 2
    hi = n_slots
    while hi > 0:
        lo = max(0, hi - _VEC_SLICE // 2)
        m = hi - lo
        sl = dev.download(vec, 2 * m - 1, np.uint32, 4 * (first + 2 * lo))[::2]
        nz = np.flatnonzero(sl)
        if len(nz):
            return lo + int(nz[-1]) + 1
        hi = lo
    return 0

def format_sources(keys: np.ndarray, pos: np.ndarray, k: int, srcs, tagged: bool) -> bytes:
    """uniq rows whose pos point into one or several sources (FastaSource /
    BatchFileSource): one merged record table in global base indices, printed
    by the host writer kman_format_uniq_mixed (no per-row Python)."""
    import ctypes
    from ctypes import byref, c_size_t, c_void_p

    from . import _native as N

    names, rec_seq, kind, base = [], [], [], []
    at = 0
    for s in srcs:
        base.append(at)
        p = s.parsed
        if p is None:
            continue
        if hasattr(s, "titles"):  # a reloaded batch file: the title is the header
            names += [t.encode("utf-8", "surrogateescape") for t in s.titles]
            kind += [1] * p.n_records
        else:
            names += list(p.names)
            kind += [0] * p.n_records
        rec_seq += (np.asarray(p.rec_seq, dtype=np.uint64) + np.uint64(at)).tolist()
        at += p.n_bases
    pos = np.asarray(pos, dtype=np.uint64)
    if tagged:
        src = (pos >> np.uint64(56)).astype(np.int64)
        pos = (pos & np.uint64((1 << 56) - 1)) + (np.asarray(base, dtype=np.uint64)[src] << np.uint64(1))
    words = np.asarray(keys).ndim == 2  # (n, W) word rows, k > 32
    keys = np.ascontiguousarray(np.asarray(keys, dtype=np.uint64).T if words else keys, dtype=np.uint64)
    pos = np.ascontiguousarray(pos, dtype=np.uint64)
    blob = b"".join(names)
    off = np.zeros(len(names) + 1, dtype=np.uint64)
    if names:
        off[1:] = np.cumsum([len(x) for x in names], dtype=np.uint64)
    rs = np.asarray(rec_seq, dtype=np.uint64)
    kd = np.asarray(kind, dtype=np.uint8)
    nb = ctypes.create_string_buffer(blob, max(1, len(blob)))
    L = N.lib()
    n = len(pos)
    if words:
        fn = L.kman_format_uniq_mixed_words
        args = (keys.ctypes.data_as(c_void_p), max(n, 1), pos.ctypes.data_as(c_void_p), n, k, nb,
                off.ctypes.data_as(c_void_p), rs.ctypes.data_as(c_void_p), kd.ctypes.data_as(c_void_p), len(names))
    else:
        fn = L.kman_format_uniq_mixed
        args = (keys.ctypes.data_as(c_void_p), pos.ctypes.data_as(c_void_p), n, k, nb,
                off.ctypes.data_as(c_void_p), rs.ctypes.data_as(c_void_p), kd.ctypes.data_as(c_void_p), len(names))
    used = c_size_t(0)
    rc = fn(*args, None, 0, byref(used), engine.host_threads())
    if rc not in (N.KMAN_OK, N.KMAN_ECAP):
        raise RuntimeError("kman_format_uniq_mixed failed (%d)" % rc)
    buf = ctypes.create_string_buffer(max(1, used.value))
    rc = fn(*args, buf, used.value, byref(used), engine.host_threads())
    if rc != N.KMAN_OK:
        raise RuntimeError("kman_format_uniq_mixed failed (%d)" % rc)
    return buf.raw[:used.value]


class KJoinerThreading(KJoiner):
    """Same surface as the reference's parallel joiner (join.py:394-480);
    ``threads`` and ``batch_size`` are accepted (the GPU join has no host
    threads to spread) — the reference's own parallel path returns wrong
    counts (§A-3), the single-thread result is the contract."""

    _threads = 1
    __batch_size = 10
    __doSort = False

    @property
    def doSort(self) -> bool:
        return self.__doSort

    @doSort.setter
    def doSort(self, doSort) -> None:
        if type(doSort) is not bool:
            raise AssertionError
        self.__doSort = doSort

    @property
    def threads(self) -> int:
        return self._threads

    @threads.setter
    def threads(self, t) -> None:
        self._threads = max(1, min(int(t), os.cpu_count() or 1))

    @property
    def batch_size(self) -> int:
        return self.__batch_size

    @batch_size.setter
    def batch_size(self, batch_size) -> None:
        if type(batch_size) is not int or batch_size < 2:
            raise AssertionError
        self.__batch_size = batch_size

    @property
    def tmp(self):
        if getattr(self, "_tmp", None) is None:
            self._tmp = tempfile.TemporaryDirectory(prefix="kmermaidJoin")
        return self._tmp
