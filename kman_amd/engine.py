"""Device-side engine: FASTA bytes -> parse -> extract -> sort -> count/uniq.

Thin Python orchestration over the C ABI (``_native``).  All per-base and
per-k-mer arithmetic runs in the gfx950 kernels of libkman.so; Python only
moves handles, sizes and the (small) record-name table.

The mapping to the reference (kmermaid 1.0.0):

=====================  ==========================================  ============================
engine function        reference                                   kernel(s)
=====================  ==========================================  ============================
``parse``              SmartFastaParser.parse, parsers.py:86-128   parse_reduce/scan/emit
``record names``       record[0].split(" ")[0], batcher.py:551     host (names only)
``extract``            Sequence.yield_kmers, seq.py:285-328        extract_kernel
``sort``               Batch.sorted, batch.py:156-168              onesweep_pass x P
``count``              Crawler.do_batch + join_sequence_count      rle_count_kernel
``uniq``               Crawler.do_batch + join_unique              rle_uniq_kernel
``format_*``           join.py:262,284 / seq.py:489-495            host threads (C++)
=====================  ==========================================  ============================
"""

from __future__ import annotations

import ctypes
import os
from ctypes import byref, c_int, c_size_t, c_uint32, c_uint64, c_void_p
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np

from . import _native as N
from . import phases

MAX_K = 32       # 2-bit keys in one u64 (the region / prefix-split paths)
MAX_K_WIDE = 64  # k <= 64: kman_extract_wide rolls the two words of a key; beyond, kman_extract_words


def host_threads() -> int:
    n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("KMAN_HOST_THREADS", "16"))))


class DeviceBuffer:
    """A device allocation owned by a :class:`Device`."""

    __slots__ = ("dev", "ptr", "nbytes")

    def __init__(self, dev: "Device", nbytes: int):
        self.dev = dev
        p = c_void_p()
        N.check(dev.ctx, N.lib().kman_malloc(dev.ctx, byref(p), max(1, int(nbytes))), "kman_malloc(%d)" % nbytes)
        self.ptr = p.value
        self.nbytes = int(nbytes)

    def free(self) -> None:
        if self.ptr and self.dev is not None and self.dev.ctx:
            N.lib().kman_free(self.dev.ctx, c_void_p(self.ptr))
        self.ptr = None

    def __del__(self):  # pragma: no cover - best effort at teardown
        try:
            self.free()
        except Exception:
            pass

    def offset(self, nbytes: int) -> int:
        return self.ptr + int(nbytes)


class Device:
    """One HIP context (stream, look-back scratch) on one GPU."""

    def __init__(self, device: int = 0):
        L = N.lib()
        ctx = c_void_p()
        rc = L.kman_create(int(device), byref(ctx))
        if rc != N.KMAN_OK:
            raise RuntimeError(
                "kman_create(device=%d) failed (%d): no usable MI355X/HIP device (%d visible)"
                % (device, rc, N.device_count())
            )
        self.ctx = ctx.value
        self.index = device
        self._fmt = None  # (cap, pinned stages) of the pipelined writer and the file loader
        phases.mark("device_init")

    def pinned_stages(self, cap: int, nb: int):
        """nb pinned host stages of >= cap bytes, kept across calls (a pinned
        allocation of a few hundred MB costs tens of ms: per call it was a
        large part of a bounded write): the pipelined writer's D2H stages and
        the chunked file loader's H2D stages.  Device memory is not held."""
        if self._fmt is not None and self._fmt[0] >= cap and len(self._fmt[1]) >= nb:
            return self._fmt[1]
        self._free_fmt()
        L = N.lib()
        stages = []
        try:
            for _ in range(nb):
                hp = c_void_p()
                N.check(self.ctx, L.kman_host_alloc(self.ctx, byref(hp), cap), "kman_host_alloc")
                stages.append(hp)
        except Exception:
            for hp in stages:
                L.kman_host_free(self.ctx, hp)
            raise
        self._fmt = (cap, stages)
        return stages

    def _free_fmt(self) -> None:
        if self._fmt is not None and self.ctx:
            L = N.lib()
            L.kman_copy_sync(self.ctx)
            for hp in self._fmt[1]:
                L.kman_host_free(self.ctx, hp)
        self._fmt = None

    def close(self) -> None:
        if self.ctx:
            self._free_fmt()
            N.lib().kman_destroy(c_void_p(self.ctx))
            self.ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # -- memory
    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def upload(self, buf: DeviceBuffer, data, offset: int = 0) -> None:
        mv = memoryview(data).cast("B")
        if offset + mv.nbytes > buf.nbytes:
            raise ValueError("upload overflows the device buffer")
        src = (ctypes.c_char * mv.nbytes).from_buffer_copy(mv) if mv.readonly else (ctypes.c_char * mv.nbytes).from_buffer(mv)
        N.check(self.ctx, N.lib().kman_memcpy_h2d(self.ctx, c_void_p(buf.ptr + offset), src, mv.nbytes), "h2d")

    def download(self, buf: DeviceBuffer, count: int, dtype, offset: int = 0) -> np.ndarray:
        out = np.empty(int(count), dtype=dtype)
        if out.nbytes:
            N.check(
                self.ctx,
                N.lib().kman_memcpy_d2h(self.ctx, out.ctypes.data_as(c_void_p), c_void_p(buf.ptr + offset), out.nbytes),
                "d2h",
            )
        return out

    def memset(self, buf: DeviceBuffer, value: int, nbytes: int, offset: int = 0) -> None:
        N.check(self.ctx, N.lib().kman_memset(self.ctx, c_void_p(buf.ptr + offset), value, nbytes), "memset")

    def sync(self) -> None:
        N.check(self.ctx, N.lib().kman_sync(self.ctx), "sync")


_DEFAULT: Optional[Device] = None


def default_device() -> Device:
    """Process-wide device (LOCAL_RANK when launched one process per GPU)."""
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = Device(int(os.environ.get("KMAN_DEVICE", os.environ.get("LOCAL_RANK", "0"))))
    return _DEFAULT


# --------------------------------------------------------------------- parse


def _title_name(text: bytes, hdr: int) -> bytes:
    """``title = line[1:].rstrip()``; ``name = title.split(" ")[0]``.

    parsers.py:85 and batcher.py:551.  Decoded like the reference's text-mode
    file (UTF-8), so Python's own rstrip/split semantics apply verbatim."""
    i = hdr + 1
    n = len(text)
    j = i
    # universal newlines: the header line ends at \n or \r
    while j < n and text[j] != 0x0A and text[j] != 0x0D:
        j += 1
    title = text[i:j].decode("utf-8", errors="surrogateescape").rstrip()
    return title.split(" ")[0].encode("utf-8", errors="surrogateescape")


@dataclass
class Parsed:
    dev: Device
    codes: DeviceBuffer  # n_bases codes + 64 pad (see include/kman.h)
    n_bases: int
    n_records: int
    rec_hdr: np.ndarray  # u64 byte offset of each '>'
    rec_seq: np.ndarray  # u64 first base index of each record
    names: List[bytes]
    names_blob: bytes
    name_off: np.ndarray  # u64, len n_records + 1

    def record_of(self, base: int) -> int:
        return int(np.searchsorted(self.rec_seq, base, side="right")) - 1

    def free(self) -> None:
        self.codes.free()


def parse(dev: Device, text: bytes) -> Parsed:
    """FASTA bytes -> device codes + record table (kman_parse_fasta)."""
    n = len(text)
    if n == 0:
        raise AssertionError("premature end of file or empty file")
    L = N.lib()
    d_text = dev.alloc(n + 64)
    codes = dev.alloc(n + 64)
    try:
        dev.upload(d_text, text)
        phases.mark("h2d")
        # record capacity: one record per 2 bytes at most ('>' + terminator)
        cap = n // 2 + 1
        d_hdr = dev.alloc(8 * cap)
        d_seq = dev.alloc(8 * cap)
        info = N.ParseInfo()
        rc = L.kman_parse_fasta(dev.ctx, c_void_p(d_text.ptr), n, c_void_p(codes.ptr), c_void_p(d_hdr.ptr),
                                c_void_p(d_seq.ptr), cap, byref(info))
        N.check(dev.ctx, rc, "kman_parse_fasta")
        R = int(info.n_records)
        rec_hdr = dev.download(d_hdr, R, np.uint64)
        rec_seq = dev.download(d_seq, R, np.uint64)
        d_hdr.free()
        d_seq.free()
    finally:
        d_text.free()
    names = [_title_name(text, int(h)) for h in rec_hdr]
    name_off = np.zeros(R + 1, dtype=np.uint64)
    if R:
        name_off[1:] = np.cumsum([len(x) for x in names], dtype=np.uint64)
    phases.mark("parse")
    return Parsed(dev, codes, int(info.n_bases), R, rec_hdr, rec_seq, names, b"".join(names), name_off)


def parse_file(dev: Device, path: str) -> Parsed:
    """kman_parse_fasta of a FASTA file (batcher.py:480 reads it whole).  A
    plain file is read in _FMT_SLICE chunks straight into two pinned stages,
    each chunk's H2D (on the copy stream) running while the next chunk is
    read, so the text crosses host memory once and no pageable copy is made;
    the record names come from the file's header lines (mmap).  Gzip input
    is inflated into memory and parsed from there (read_input + parse)."""
    if path.endswith(".gz"):
        return parse(dev, read_input(path))
    import mmap

    L = N.lib()
    with open(path, "rb", buffering=0) as fh:
        n = os.fstat(fh.fileno()).st_size
        if n == 0:
            raise AssertionError("premature end of file or empty file")
        d_text = dev.alloc(n + 64)
        codes = dev.alloc(n + 64)
        try:
            stages = dev.pinned_stages(_FMT_SLICE + 16, 2)
            at, i = 0, 0
            while at < n:
                b, m = i % 2, min(_FMT_SLICE, n - at)
                mv = memoryview((ctypes.c_char * m).from_address(stages[b].value)).cast("B")
                got = 0
                while got < m:
                    r = fh.readinto(mv[got:])
                    if not r:
                        raise OSError("%s: short read at byte %d of %d" % (path, at + got, n))
                    got += r
                # the chunk before this one is out of its stage (and stage b's
                # previous chunk long since): then this chunk's copy is queued
                N.check(dev.ctx, L.kman_copy_sync(dev.ctx), "kman_copy_sync")
                N.check(dev.ctx, L.kman_copy_h2d_async(dev.ctx, c_void_p(d_text.ptr + at), stages[b], m, b),
                        "kman_copy_h2d_async")
                at += m
                i += 1
            N.check(dev.ctx, L.kman_copy_sync(dev.ctx), "kman_copy_sync")
            phases.mark("file_read+h2d")
            cap = n // 2 + 1
            d_hdr = dev.alloc(8 * cap)
            d_seq = dev.alloc(8 * cap)
            try:
                info = N.ParseInfo()
                N.check(dev.ctx, L.kman_parse_fasta(dev.ctx, c_void_p(d_text.ptr), n, c_void_p(codes.ptr),
                                                    c_void_p(d_hdr.ptr), c_void_p(d_seq.ptr), cap, byref(info)),
                        "kman_parse_fasta")
                R = int(info.n_records)
                rec_hdr = dev.download(d_hdr, R, np.uint64)
                rec_seq = dev.download(d_seq, R, np.uint64)
            finally:
                d_hdr.free()
                d_seq.free()
        except BaseException:
            codes.free()
            raise
        finally:
            d_text.free()
        mm = mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ)
        try:
            names = [_title_name(mm, int(h)) for h in rec_hdr]
        finally:
            mm.close()
    name_off = np.zeros(R + 1, dtype=np.uint64)
    if R:
        name_off[1:] = np.cumsum([len(x) for x in names], dtype=np.uint64)
    phases.mark("parse")
    return Parsed(dev, codes, int(info.n_bases), R, rec_hdr, rec_seq, names, b"".join(names), name_off)


def check_empty_names(p: Parsed, k: int) -> None:
    """The reference re-reads every k-mer header through
    ``SequenceCoords.from_str`` (seq.py:106-127, via batch.py:170-186) whose
    regex needs a non-empty record name: a record with an empty name that
    yields any k-mer raises AssertionError before any output is written."""
    for r, nm in enumerate(p.names):
        if nm:
            continue
        b = int(p.rec_seq[r])
        e = int(p.rec_seq[r + 1]) if r + 1 < p.n_records else p.n_bases
        if e - b < k:
            continue
        st = first_window(p.dev.download(p.codes, e - b, np.uint8, offset=b), k)
        if st >= 0:
            raise AssertionError("incompatible string: :%d-%d:+" % (st, st + k))


def first_window(codes: np.ndarray, k: int) -> int:
    """Start of the first run of k ACGT codes (code & 7 < 4) in one record's
    codes, or -1 (vectorised: run starts and ends of the valid positions)."""
    ok = (np.asarray(codes) & 7) < 4
    if len(ok) < k or not ok.any():
        return -1
    d = np.diff(np.concatenate([[0], ok.view(np.int8), [0]]))
    starts = np.nonzero(d == 1)[0]
    ends = np.nonzero(d == -1)[0]
    long = np.nonzero(ends - starts >= k)[0]
    return int(starts[long[0]]) if len(long) else -1


# ------------------------------------------------------------------- extract


@dataclass
class Kmers:
    """k-mer keys (+ pos payload) in the reference's stream order."""

    keys: DeviceBuffer
    alt: DeviceBuffer
    pos: Optional[DeviceBuffer]
    pos_alt: Optional[DeviceBuffer]
    pos_bytes: int
    n: int
    k: int
    hist: DeviceBuffer
    sorted: bool = False
    # histogram plan of kman_extract: bits [lo_bit, 2k) (kman_split_bits);
    # hist_valid False = no usable histogram (sort computes its own)
    lo_bit: int = 0
    hist_valid: bool = False
    prefix_sorted: bool = False  # keys stably sorted by bits [lo_bit, 2k) (kman_extract_sorted)

    def free(self) -> None:
        for b in (self.keys, self.alt, self.pos, self.pos_alt, self.hist):
            if b is not None:
                b.free()


def flags_for(rc: bool, want_pos: bool, canonical: bool = False, mixed: bool = False) -> int:
    """kman_extract flags; mixed (with canonical): the keys through the
    bijection of KMAN_MIXED -- spectra only, the keys are not printed."""
    return ((N.KMAN_RC if rc else 0) | (N.KMAN_WANT_POS if want_pos else 0) | (N.KMAN_CANONICAL if canonical else 0)
            | (N.KMAN_MIXED if canonical and mixed else 0))


def count_kmers(p: Parsed, k: int, rc: bool, canonical: bool = False) -> int:
    _check_k(k, wide=True)
    out = c_uint64(0)
    if k > MAX_K_WIDE:
        N.check(p.dev.ctx, N.lib().kman_extract_words(p.dev.ctx, c_void_p(p.codes.ptr), p.n_bases, k,
                                                      flags_for(rc, False, canonical), None, 0, None, 0, 0,
                                                      byref(out)), "kman_extract_words")
        return int(out.value)
    if k > MAX_K:
        N.check(p.dev.ctx, N.lib().kman_extract_wide(p.dev.ctx, c_void_p(p.codes.ptr), p.n_bases, k,
                                                     flags_for(rc, False, canonical), None, None, None, 0, 0,
                                                     byref(out)), "kman_extract_wide")
        return int(out.value)
    N.check(p.dev.ctx, N.lib().kman_count_kmers(p.dev.ctx, c_void_p(p.codes.ptr), p.n_bases, k,
                                                 flags_for(rc, False, canonical), byref(out)), "kman_count_kmers")
    return int(out.value)


def _check_k(k: int, wide: bool = False) -> None:
    """batcher.py:477-478 (k <= 1 raises AssertionError); a path that packs a
    k-mer in one 64-bit key (region / prefix-split / multi-GPU) takes
    k <= 32, the word-key path (wide) every k."""
    if k <= 1:
        raise AssertionError("k must be >= 1, got %d instead." % k)
    if not wide and k > MAX_K:
        raise NotImplementedError("k=%d: this path packs k-mers in one 64-bit key (k <= %d); the word-key path "
                                  "takes larger k" % (k, MAX_K))


def extract(p: Parsed, k: int, rc: bool, want_pos: bool, canonical: bool = False) -> Kmers:
    """kman_extract: keys (+ pos) in stream order, plus the radix histograms."""
    _check_k(k)
    dev = p.dev
    L = N.lib()
    bound = p.n_bases * (2 if rc and not canonical else 1)
    n = max(bound, 1)
    pos_bytes = 4 if 2 * p.n_bases <= 0xFFFFFFFF else 8
    keys = dev.alloc(8 * n)
    alt = dev.alloc(8 * n)
    pos = dev.alloc(pos_bytes * n) if want_pos else None
    pos_alt = dev.alloc(pos_bytes * n) if want_pos else None
    hist = dev.alloc(8 * 256 * 8)
    dev.memset(hist, 0, 8 * 256 * 8)
    out = c_uint64(0)
    lo = split_bits(bound, 2 * k)
    rc_ = L.kman_extract(dev.ctx, c_void_p(p.codes.ptr), p.n_bases, k,
                         flags_for(rc, want_pos, canonical) | N.KMAN_HIST_LO(lo),
                         c_void_p(keys.ptr), c_void_p(pos.ptr if pos else None), pos_bytes, bound,
                         c_void_p(hist.ptr), byref(out))
    N.check(dev.ctx, rc_, "kman_extract")
    return Kmers(keys, alt, pos, pos_alt, pos_bytes if want_pos else 0, int(out.value), k, hist, lo_bit=lo,
                 hist_valid=True)


def extract_sorted(p: Parsed, k: int, rc: bool, want_pos: bool, canonical: bool = False) -> Kmers:
    """kman_extract_sorted: the k-mers already stably sorted by their prefix
    bits [lo, 2k) (first prefix pass fused into the extraction)."""
    _check_k(k)
    dev = p.dev
    L = N.lib()
    bound = p.n_bases * (2 if rc and not canonical else 1)
    n = max(bound, 1)
    pos_bytes = 4 if 2 * p.n_bases <= 0xFFFFFFFF else 8
    keys, alt = dev.alloc(8 * n), dev.alloc(8 * n)
    pos = dev.alloc(pos_bytes * n) if want_pos else None
    pos_alt = dev.alloc(pos_bytes * n) if want_pos else None
    lo = split_bits(bound, 2 * k)
    out, res = c_uint64(0), c_int(0)
    N.check(dev.ctx, L.kman_extract_sorted(dev.ctx, c_void_p(p.codes.ptr), p.n_bases, k,
                                           flags_for(rc, want_pos, canonical), lo,
                                           c_void_p(keys.ptr), c_void_p(alt.ptr),
                                           c_void_p(pos.ptr if pos else None), c_void_p(pos_alt.ptr if pos else None),
                                           pos_bytes, bound, byref(out), byref(res)), "kman_extract_sorted")
    if res.value:
        keys, alt = alt, keys
        pos, pos_alt = pos_alt, pos
    return Kmers(keys, alt, pos, pos_alt, pos_bytes if want_pos else 0, int(out.value), k, dev.alloc(8), lo_bit=lo,
                 prefix_sorted=True)


def split_bits(n: int, key_bits: int) -> int:
    """kman_split_bits: low bit of the prefix the global passes sort by."""
    lo = ctypes.c_uint32(0)
    if N.lib().kman_split_bits(max(int(n), 0), key_bits, byref(lo)) != N.KMAN_OK:
        raise ValueError("bad key_bits %d" % key_bits)
    return int(lo.value)


def _sort_prefix(km: Kmers, dev: Device, key_bits: int) -> None:
    """kman_sort_range over bits [km.lo_bit, key_bits): a stable sort by the
    prefix; km.keys / km.pos then hold the prefix-sorted data."""
    if km.prefix_sorted:
        return
    res = c_int(0)
    hist = c_void_p(km.hist.ptr) if km.hist_valid and km.hist is not None else c_void_p(None)
    rc = N.lib().kman_sort_range(dev.ctx, c_void_p(km.keys.ptr), c_void_p(km.alt.ptr),
                                 c_void_p(km.pos.ptr if km.pos else None),
                                 c_void_p(km.pos_alt.ptr if km.pos_alt else None), km.pos_bytes, km.n, km.lo_bit,
                                 key_bits, hist, byref(res))
    N.check(dev.ctx, rc, "kman_sort_range")
    if res.value:
        km.keys, km.alt = km.alt, km.keys
        km.pos, km.pos_alt = km.pos_alt, km.pos
    km.prefix_sorted = True


def _finish(km: Kmers, dev: Device, key_bits: int, mode: int, okeys=None, ovals=None, ob: int = 0) -> int:
    out = c_uint64(0)
    N.check(dev.ctx, N.lib().kman_finish(dev.ctx, c_void_p(km.keys.ptr), c_void_p(km.alt.ptr),
                                         c_void_p(km.pos.ptr if km.pos else None),
                                         c_void_p(km.pos_alt.ptr if km.pos_alt else None), km.pos_bytes, km.n,
                                         key_bits, km.lo_bit, mode, c_void_p(okeys.ptr if okeys else None),
                                         c_void_p(ovals.ptr if ovals else None), ob, byref(out)), "kman_finish")
    return int(out.value)


def sort(km: Kmers, dev: Device) -> None:
    """Stable sort of km.keys (+ km.pos) by key, Batch.sorted (batch.py:156-168):
    kman_sort_range over the prefix bits, then kman_finish(SORT) in LDS."""
    if km.sorted:
        return
    if km.n > 1:
        _sort_prefix(km, dev, 2 * km.k)
        _finish(km, dev, 2 * km.k, N.KMAN_FINISH_SORT)
    km.sorted = True


@dataclass
class CountResult:
    ukeys: DeviceBuffer
    counts: DeviceBuffer
    count_bytes: int
    n: int
    k: int


def rle_count(km: Kmers, dev: Device) -> CountResult:
    """(key, group size) per distinct key.  Sorted input: kman_rle_count;
    unsorted: the prefix sort + kman_finish(COUNT) (km is consumed)."""
    cb = 4 if km.n <= 0xFFFFFFFF else 8
    ukeys = dev.alloc(8 * max(km.n, 1))
    counts = dev.alloc(cb * max(km.n, 1))
    if not km.sorted:
        _sort_prefix(km, dev, 2 * km.k)
        n = _finish(km, dev, 2 * km.k, N.KMAN_FINISH_COUNT, ukeys, counts, cb)
        return CountResult(ukeys, counts, cb, n, km.k)
    out = c_uint64(0)
    N.check(dev.ctx, N.lib().kman_rle_count(dev.ctx, c_void_p(km.keys.ptr), km.n, c_void_p(ukeys.ptr),
                                             c_void_p(counts.ptr), cb, byref(out)), "kman_rle_count")
    return CountResult(ukeys, counts, cb, int(out.value), km.k)


@dataclass
class UniqResult:
    keys: DeviceBuffer
    pos: DeviceBuffer
    pos_bytes: int
    n: int
    k: int


def rle_uniq(km: Kmers, dev: Device) -> UniqResult:
    if km.pos is None:
        raise ValueError("uniq needs the pos payload (extract with want_pos=True)")
    okeys = dev.alloc(8 * max(km.n, 1))
    opos = dev.alloc(km.pos_bytes * max(km.n, 1))
    if not km.sorted:
        _sort_prefix(km, dev, 2 * km.k)
        n = _finish(km, dev, 2 * km.k, N.KMAN_FINISH_UNIQ, okeys, opos, km.pos_bytes)
        return UniqResult(okeys, opos, km.pos_bytes, n, km.k)
    out = c_uint64(0)
    N.check(dev.ctx, N.lib().kman_rle_uniq(dev.ctx, c_void_p(km.keys.ptr), c_void_p(km.pos.ptr), km.pos_bytes,
                                            km.n, c_void_p(okeys.ptr), c_void_p(opos.ptr), byref(out)),
            "kman_rle_uniq")
    return UniqResult(okeys, opos, km.pos_bytes, int(out.value), km.k)


def groups(p: Parsed, k: int, rc: bool, mode: str, canonical: bool = False, mixed: bool = False):
    """kman_groups: count / uniq of the whole stream straight from the codes
    (region.hip).  Returns a CountResult / UniqResult, or None when the input
    is outside the region path (kman_groups_plan / a region overflow said
    KMAN_EFALLBACK): the caller then runs extract_sorted + rle_*."""
    L, dev = N.lib(), p.dev
    m = N.KMAN_FINISH_UNIQ if mode == "uniq" else N.KMAN_FINISH_COUNT
    flags = flags_for(rc, mode == "uniq", canonical, mixed)
    wb = c_uint64(0)
    rc_ = L.kman_groups_plan(p.n_bases, k, flags, m, byref(wb))
    if rc_ == N.KMAN_EFALLBACK:
        return None
    N.check(dev.ctx, rc_, "kman_groups_plan")
    cap = max(1, p.n_bases * (2 if rc and not canonical else 1))
    vb = (4 if 2 * p.n_bases <= 0xFFFFFFFF else 8) if mode == "uniq" else (4 if cap <= 0xFFFFFFFF else 8)
    work = dev.alloc(int(wb.value))
    okeys = dev.alloc(8 * cap)
    ovals = dev.alloc(vb * cap)
    phases.mark("groups_alloc")
    nk, no = c_uint64(0), c_uint64(0)
    try:
        rc_ = L.kman_groups(dev.ctx, c_void_p(p.codes.ptr), p.n_bases, k, flags, m, c_void_p(work.ptr), wb.value,
                            c_void_p(okeys.ptr), c_void_p(ovals.ptr), vb, byref(nk), byref(no))
    finally:
        work.free()
    phases.mark("groups_kernels")
    if rc_ == N.KMAN_EFALLBACK:
        okeys.free()
        ovals.free()
        return None
    N.check(dev.ctx, rc_, "kman_groups")
    if mode == "uniq":
        return UniqResult(okeys, ovals, vb, int(no.value), k)
    return CountResult(okeys, ovals, vb, int(no.value), k)


def mem_info(dev: Device) -> Tuple[int, int]:
    """(free, total) HBM bytes of the device (kman_mem_info)."""
    f, t = c_size_t(0), c_size_t(0)
    N.check(dev.ctx, N.lib().kman_mem_info(dev.ctx, byref(f), byref(t)), "kman_mem_info")
    return int(f.value), int(t.value)


def _prefix_hist_into(p: Parsed, k: int, rc: bool, h: DeviceBuffer) -> Tuple[np.ndarray, int]:
    n = c_uint64(0)
    N.check(p.dev.ctx, N.lib().kman_kmer_prefix_hist(p.dev.ctx, c_void_p(p.codes.ptr), p.n_bases, k,
                                                      N.KMAN_RC if rc else 0, c_void_p(h.ptr), byref(n)),
            "kman_kmer_prefix_hist")
    bins = 256 if 2 * k >= 8 else 1 << (2 * k)
    return p.dev.download(h, bins, np.uint64), int(n.value)


def prefix_hist(p: Parsed, k: int, rc: bool) -> Tuple[np.ndarray, int]:
    """Histogram of the top 8 key bits of the stream (kman_kmer_prefix_hist):
    4^k bins when 2k < 8.  Returns (hist, n_kmers)."""
    _check_k(k)
    h = p.dev.alloc(8 * 256)
    try:
        return _prefix_hist_into(p, k, rc, h)
    finally:
        h.free()


def key_ranges(hist: np.ndarray, k: int, max_keys: int, count=None) -> List[Tuple[int, int, int]]:
    """Consecutive top-8-bit prefixes grouped into key ranges of at most
    max_keys k-mers: [(key_lo, key_hi, n)] in key order, empty ranges dropped.
    The batches of a multi-batch join (join.py:63-130) cut by key instead of
    by stream position: their n-way merge is then their concatenation.  A
    prefix holding more than max_keys k-mers (repeats, poly-A) is bisected
    by key with count(lo, hi) -> k-mers in [lo, hi] until its pieces fit;
    only one key value repeated more than max_keys times cannot be cut."""
    shift = max(0, 2 * k - 8)
    out, lo, acc = [], 0, 0

    def split(a, b, c):
        if c <= max_keys:
            return [(a, b, c)] if c else []
        if a == b or count is None:
            raise MemoryError("%d k-mers in key range [%x, %x]: more than a batch of %d" % (c, a, b, max_keys))
        m = (a + b) // 2
        c0 = count(a, m)
        return split(a, m, c0) + split(m + 1, b, c - c0)

    for b, c in enumerate(hist.tolist()):
        if c > max_keys:
            if acc:
                out.append((lo << shift, (b << shift) - 1, acc))
            out.extend(split(b << shift, ((b + 1) << shift) - 1, c))
            lo, acc = b + 1, 0
            continue
        if acc and acc + c > max_keys:
            out.append((lo << shift, (b << shift) - 1, acc))
            lo, acc = b, 0
        acc += c
    if acc:
        out.append((lo << shift, (len(hist) << shift) - 1, acc))
    return out


class _At:
    """A device pointer inside a buffer (an output slice) for _finish."""

    def __init__(self, buf: DeviceBuffer, offset: int):
        self.ptr = buf.ptr + int(offset)


class RangedJoin:
    """Multi-batch device join (BASELINE config 3): count / uniq of a stream
    whose k-mers do not fit the device at once.  The stream is cut into key
    ranges of at most max_keys k-mers (prefix_hist + key_ranges); each range
    is extracted from the resident codes (kman_extract_range, stream order),
    prefix-sorted (kman_sort_range) and finished in LDS (kman_finish), its
    output appended to the global output, which is therefore in key order.
    Same results as groups() / extract_sorted + rle_* (join.py:95-130,
    244-285 over batch.py:156-168).  Every buffer is allocated here, once:
    ``step()`` re-plans (prefix histogram) and runs the batches."""

    def __init__(self, p: Parsed, k: int, rc: bool, mode: str, max_keys: Optional[int] = None):
        _check_k(k)
        self.p, self.k, self.rc, self.mode = p, k, rc, mode
        dev = self.dev = p.dev
        self.want_pos = mode == "uniq"
        self._bufs = []
        self.phist = self._alloc(8 * 256)
        hist, n = _prefix_hist_into(p, k, rc, self.phist)
        self.n_kmers = n
        self.pos_bytes = 4 if 2 * p.n_bases <= 0xFFFFFFFF else 8
        self.vb = self.pos_bytes if self.want_pos else (4 if n <= 0xFFFFFFFF else 8)
        per_key = 16 + (2 * self.pos_bytes if self.want_pos else 0)
        if max_keys is None:
            free, _ = mem_info(dev)
            max_keys = max(1 << 20, (int(free * 0.85) - (8 + self.vb) * n) // per_key)
        self.max_keys = int(max_keys)
        self.ranges = key_ranges(hist, k, self.max_keys, self._count_range)
        self.cap = max([r[2] for r in self.ranges] + [1])
        self.okeys = self._alloc(8 * max(n, 1))
        self.ovals = self._alloc(self.vb * max(n, 1))
        self.keys, self.alt = self._alloc(8 * self.cap), self._alloc(8 * self.cap)
        self.pos = self._alloc(self.pos_bytes * self.cap) if self.want_pos else None
        self.pos_alt = self._alloc(self.pos_bytes * self.cap) if self.want_pos else None
        self.hbuf = self._alloc(8 * 256 * 8)
        self.n_out = 0

    def _count_range(self, lo: int, hi: int) -> int:
        """k-mers with keys in [lo, hi] (kman_extract_range with no capacity:
        counted, nothing written)."""
        got = c_uint64(0)
        rc = N.lib().kman_extract_range(self.dev.ctx, c_void_p(self.p.codes.ptr), self.p.n_bases, self.k,
                                        flags_for(self.rc, False), lo, hi, None, None, 4, 0, None, byref(got))
        if rc not in (N.KMAN_OK, N.KMAN_ECAP):
            N.check(self.dev.ctx, rc, "kman_extract_range")
        return int(got.value)

    def _alloc(self, nbytes: int) -> DeviceBuffer:
        try:
            b = self.dev.alloc(nbytes)
        except BaseException:
            self.free()
            raise
        self._bufs.append(b)
        return b

    def step(self) -> int:
        """One whole join: plan the key ranges, then extract + sort + finish
        each range into the output.  Returns the number of k-mers joined."""
        dev, L, k, p = self.dev, N.lib(), self.k, self.p
        hist, n = _prefix_hist_into(p, k, self.rc, self.phist)
        ranges = self.ranges
        if n != self.n_kmers:
            raise RuntimeError("the stream changed under a planned RangedJoin")
        flags = flags_for(self.rc, self.want_pos)
        fmode = N.KMAN_FINISH_UNIQ if self.want_pos else N.KMAN_FINISH_COUNT
        shift = max(0, 2 * k - 8)
        vb, pb = self.vb, self.pos_bytes
        total = 0
        for lo_key, hi_key, nr in ranges:
            # the range's keys fill (hi - lo + 1) of the len(hist) prefixes:
            # segment bits as for a stream that dense over the whole key space
            lo = split_bits(nr * (1 << (2 * k)) // (hi_key - lo_key + 1), 2 * k)
            dev.memset(self.hbuf, 0, 8 * 256 * 8)
            got = c_uint64(0)
            N.check(dev.ctx, L.kman_extract_range(dev.ctx, c_void_p(p.codes.ptr), p.n_bases, k,
                                                  flags | N.KMAN_HIST_LO(lo), lo_key, hi_key,
                                                  c_void_p(self.keys.ptr),
                                                  c_void_p(self.pos.ptr if self.pos else None), pb, self.cap,
                                                  c_void_p(self.hbuf.ptr), byref(got)), "kman_extract_range")
            if int(got.value) != nr:
                raise RuntimeError("key range [%x, %x]: %d k-mers extracted, histogram said %d"
                                   % (lo_key, hi_key, got.value, nr))
            km = Kmers(self.keys, self.alt, self.pos, self.pos_alt, pb if self.want_pos else 0, nr, k, self.hbuf,
                       lo_bit=lo, hist_valid=True)
            _sort_prefix(km, dev, 2 * k)
            total += _finish(km, dev, 2 * k, fmode, _At(self.okeys, 8 * total), _At(self.ovals, vb * total), vb)
            self.keys, self.alt, self.pos, self.pos_alt = km.keys, km.alt, km.pos, km.pos_alt
        self.n_out = total
        return n

    def result(self):
        """The output (CountResult / UniqResult); its buffers now belong to
        the caller."""
        r = (UniqResult if self.want_pos else CountResult)(self.okeys, self.ovals, self.vb, self.n_out, self.k)
        self._bufs = [b for b in self._bufs if b is not self.okeys and b is not self.ovals]
        return r

    def free(self) -> None:
        for b in self._bufs:
            b.free()
        self._bufs = []


def ranged_groups(p: Parsed, k: int, rc: bool, mode: str, max_keys: Optional[int] = None):
    """RangedJoin in one call: the CountResult / UniqResult of the stream."""
    j = RangedJoin(p, k, rc, mode, max_keys)
    try:
        j.step()
        return j.result()
    finally:
        j.free()


# ------------------------------------------------------------------ formatting


def _format(fn, *args) -> bytes:
    used = c_size_t(0)
    rc = fn(*args, None, 0, byref(used), host_threads())
    if rc not in (N.KMAN_OK, N.KMAN_ECAP):
        raise RuntimeError("formatter failed (%d)" % rc)
    buf = ctypes.create_string_buffer(max(1, used.value))
    rc = fn(*args, buf, used.value, byref(used), host_threads())
    if rc != N.KMAN_OK:
        raise RuntimeError("formatter failed (%d)" % rc)
    return buf.raw[: used.value]


def format_fasta_words(rows: np.ndarray, pos: np.ndarray, k: int, p: Parsed) -> bytes:
    """The batch-file FASTA (KMer.as_fasta, seq.py:489-495) of word-key rows
    ((n, W) host array) with headers from the record table (host writer
    kman_format_uniq_words)."""
    planes = np.ascontiguousarray(np.asarray(rows, dtype=np.uint64).T)
    n = planes.shape[1] if planes.ndim == 2 else 0
    pos = np.ascontiguousarray(pos, dtype=np.uint64)
    names = ctypes.create_string_buffer(p.names_blob, max(1, len(p.names_blob)))
    off = np.ascontiguousarray(p.name_off, dtype=np.uint64)
    rs = np.ascontiguousarray(p.rec_seq, dtype=np.uint64)
    return _format(N.lib().kman_format_uniq_words, planes.ctypes.data_as(c_void_p), max(n, 1),
                   pos.ctypes.data_as(c_void_p), 8, n, k, names, off.ctypes.data_as(c_void_p),
                   rs.ctypes.data_as(c_void_p), max(p.n_records, 1))


def format_count(ukeys: np.ndarray, counts: np.ndarray, k: int) -> bytes:
    """``"%s\\t%d\\n" % (seq, count)`` per group (join.py:283-284)."""
    ukeys = np.ascontiguousarray(ukeys, dtype=np.uint64)
    cb = counts.dtype.itemsize
    return _format(N.lib().kman_format_count, ukeys.ctypes.data_as(c_void_p),
                   np.ascontiguousarray(counts).ctypes.data_as(c_void_p), cb, len(ukeys), k)


def format_fasta(keys: np.ndarray, pos: np.ndarray, k: int, p: Parsed) -> bytes:
    """``">%s\\n%s\\n" % (header, seq)`` (join.py:262 / seq.py:495)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    pos = np.ascontiguousarray(pos)
    names = ctypes.create_string_buffer(p.names_blob, max(1, len(p.names_blob)))
    off = np.ascontiguousarray(p.name_off, dtype=np.uint64)
    rs = np.ascontiguousarray(p.rec_seq, dtype=np.uint64)
    return _format(N.lib().kman_format_uniq, keys.ctypes.data_as(c_void_p), pos.ctypes.data_as(c_void_p),
                   pos.dtype.itemsize, len(keys), k, names, off.ctypes.data_as(c_void_p),
                   rs.ctypes.data_as(c_void_p), p.n_records)


# device-side formatting: the text is built in HBM and only
# the text crosses PCIe; slices of at most _FMT_CHUNK text bytes per launch
_FMT_CHUNK = 1 << 31
_FMT_SLICE = 256 << 20  # text bytes per pipelined slice (_format_dev)
_FMT_THREADS = int(os.environ.get("KMAN_FMT_THREADS", "8"))  # host copy threads
# the format kernels write the pinned stages directly (zero-copy over PCIe)
# instead of a device slice + a copy-engine D2H: the copy engine ran a fresh
# process's first ~2 s at ~31 GB/s (8.2 ms per 256 MiB slice, then 4.2 once
# warm), the kernels' own writes reach ~54 GB/s from the first slice
# (tools/fmtcold.py: 49 GB of uniq text 1.02 s cold vs 1.76; warm 0.92 vs
# 0.88).  KMAN_FMT_ZC=0: the copy-engine pipeline.
_FMT_ZC = os.environ.get("KMAN_FMT_ZC", "1") != "0"


def _pwrite_target(sink):
    """(fd, offset) when the pipelined writer may put slices at computed
    offsets with os.pwrite -- a regular file not opened for appending (pwrite
    on an O_APPEND descriptor ignores the offset on Linux, and a pipe or a
    terminal has no offsets) -- else (None, 0): the slices are then written
    in order by the calling thread through sink.write."""
    import fcntl
    import stat

    try:
        sink.flush()
        fd = sink.fileno()
        if not stat.S_ISREG(os.fstat(fd).st_mode) or fcntl.fcntl(fd, fcntl.F_GETFL) & os.O_APPEND:
            return None, 0
        return fd, sink.tell()
    except (AttributeError, OSError, ValueError):
        return None, 0


def _format_dev(dev: Device, n: int, row_bytes: int, call, sink=None):
    """Run a kman_format_*_dev call over row slices.  call(i0, rows, d_out,
    cap, used) formats rows [i0, i0 + rows); row_bytes bounds one row.
    Returns the text (a bytearray), or, with a sink (a binary file), writes
    it there and returns None.

    Pipelined over slices of <= _FMT_SLICE text bytes through two pinned
    stages: the format kernel writes slice i straight into stage i % 2 over
    PCIe (_FMT_ZC, the default) while a pool of host threads copies slice
    i - 1 out of the other stage -- pwrite at its file offset, or memmove
    into the result.  (KMAN_FMT_ZC=0: slice i formatted into a device slice
    while slice i - 1 crosses PCIe on the copy stream, kman_copy_d2h_async,
    and slice i - 2 leaves its stage.)"""
    if n == 0:
        return None if sink is not None else bytearray()
    import concurrent.futures as cf

    L = N.lib()
    rows = max(1, min(n, _FMT_SLICE // max(1, row_bytes)))
    cap = rows * row_bytes + 16
    used = c_size_t(0)
    out, fd, base = None, None, 0
    if sink is None:
        rc_ = call(0, n, None, 0, used)  # sizing pass over every row
        if rc_ not in (N.KMAN_OK, N.KMAN_ECAP):
            N.check(dev.ctx, rc_, "kman_format_*_dev")
        out = bytearray(int(used.value))
        dst0 = ctypes.addressof((ctypes.c_char * max(1, len(out))).from_buffer(out)) if len(out) else 0
    else:
        fd, base = _pwrite_target(sink)
    NB = 2
    stages = dev.pinned_stages(max(cap, _FMT_SLICE + 16), NB)
    # (the device text slices live for this call only: held across calls
    # they would hide 2 x 256 MiB from later mem_info-based plans)
    dbufs = [] if _FMT_ZC else [dev.alloc(cap) for _ in range(NB)]
    phases.mark("fmt_buffers")
    pool = cf.ThreadPoolExecutor(max_workers=_FMT_THREADS)
    wpool = cf.ThreadPoolExecutor(max_workers=1)
    try:
        pending = [[] for _ in range(NB)]
        piece = max(1 << 20, cap // _FMT_THREADS + 1)

        def copy_piece(src, at, u):
            if out is not None:
                ctypes.memmove(dst0 + at, src, u)
            else:
                mv = memoryview((ctypes.c_char * u).from_address(src)).cast("B")
                done = 0
                while done < u:
                    done += os.pwrite(fd, mv[done:], base + at + done)

        def drain(b, at, u):
            """slice in stage b (u bytes at text offset `at`) out to the host"""
            N.check(dev.ctx, L.kman_copy_d2h_wait(dev.ctx, b), "kman_copy_d2h_wait")
            if out is None and fd is None:
                sink.write(memoryview((ctypes.c_char * u).from_address(stages[b].value)).cast("B"))
                return
            pending[b] = [pool.submit(copy_piece, stages[b].value + o, at + o, min(piece, u - o))
                          for o in range(0, u, piece)]

        at, last = 0, None
        if _FMT_ZC:
            # zero-copy: the format kernel writes slice i straight into pinned
            # stage b over PCIe (no copy engine); the host drains stage b while
            # slice i + 1 is formatted into the other stage
            for i, i0 in enumerate(range(0, n, rows)):
                b = i % NB
                for f in pending[b]:
                    f.result()
                pending[b] = []
                m = min(rows, n - i0)
                N.check(dev.ctx, call(i0, m, stages[b], cap, used), "kman_format_*_dev")
                u = int(used.value)
                if out is None and fd is None:  # a stream: one writer thread keeps the slices in order
                    mv = memoryview((ctypes.c_char * u).from_address(stages[b].value)).cast("B")
                    pending[b] = [wpool.submit(sink.write, mv)]
                else:
                    pending[b] = [pool.submit(copy_piece, stages[b].value + o, at + o, min(piece, u - o))
                                  for o in range(0, u, piece)]
                if i == 0:
                    phases.mark("fmt_first_slice")
                at += u
            for pb in pending:
                for f in pb:
                    f.result()
        else:
            for i, i0 in enumerate(range(0, n, rows)):
                b = i % NB
                for f in pending[b]:  # slice i - 2 out of stage b (its D2H finished before)
                    f.result()
                pending[b] = []
                m = min(rows, n - i0)
                N.check(dev.ctx, call(i0, m, c_void_p(dbufs[b].ptr), cap, used), "kman_format_*_dev")
                u = int(used.value)
                N.check(dev.ctx, L.kman_copy_d2h_async(dev.ctx, stages[b], c_void_p(dbufs[b].ptr), u, b),
                        "kman_copy_d2h_async")
                if last is not None:
                    drain(*last)
                    if i == 1:
                        phases.mark("fmt_first_slice")
                last = (b, at, u)
                at += u
            if last is not None:
                drain(*last)
            for pb in pending:
                for f in pb:
                    f.result()
    finally:
        pool.shutdown(wait=True)
        wpool.shutdown(wait=True)
        N.check(dev.ctx, L.kman_copy_sync(dev.ctx), "kman_copy_sync")
        for b_ in dbufs:
            b_.free()
    if out is not None:
        assert at == len(out)
        return out
    if fd is not None:
        sink.seek(base + at)
    return None


def format_count_dev(dev: Device, r: CountResult, sink=None):
    """``"%s\t%d\n" % (seq, count)`` per group (join.py:283-284), built on
    the device from the device-resident result (kman_format_count_dev)."""
    L, cb = N.lib(), r.count_bytes

    def call(i0, m, d_out, cap, used):
        return L.kman_format_count_dev(dev.ctx, c_void_p(r.ukeys.ptr + 8 * i0), c_void_p(r.counts.ptr + cb * i0), cb,
                                       m, r.k, d_out, cap, byref(used))

    return _format_dev(dev, r.n, r.k + 2 + (10 if cb == 4 else 20), call, sink)


class DeviceNames:
    """The record table of a Parsed input on the device (names blob, name
    offsets, first base of each record) for kman_format_uniq_dev."""

    def __init__(self, p: Parsed):
        dev = p.dev
        self.names = dev.alloc(max(16, len(p.names_blob)))
        self.off = dev.alloc(8 * (p.n_records + 1))
        self.rec = dev.alloc(8 * max(1, p.n_records))
        if p.names_blob:
            dev.upload(self.names, p.names_blob)
        dev.upload(self.off, np.ascontiguousarray(p.name_off, dtype=np.uint64))
        if p.n_records:
            dev.upload(self.rec, np.ascontiguousarray(p.rec_seq, dtype=np.uint64))
        self.n_records = p.n_records
        self.max_name = int(np.diff(p.name_off).max()) if p.n_records else 0
        self.n_bases = p.n_bases

    def free(self) -> None:
        for b in (self.names, self.off, self.rec):
            b.free()


def format_uniq_dev(p: Parsed, r: UniqResult, sink=None):
    """``">%s\n%s\n" % (header, seq)`` (join.py:262 / seq.py:495), built on
    the device (kman_format_uniq_dev)."""
    dev, L, pb = p.dev, N.lib(), r.pos_bytes
    nm = DeviceNames(p)
    try:
        D = len(str(p.n_bases + r.k))

        def call(i0, m, d_out, cap, used):
            return L.kman_format_uniq_dev(dev.ctx, c_void_p(r.keys.ptr + 8 * i0), c_void_p(r.pos.ptr + pb * i0), pb,
                                          m, r.k, c_void_p(nm.names.ptr), c_void_p(nm.off.ptr), c_void_p(nm.rec.ptr),
                                          nm.n_records, d_out, cap, byref(used))

        return _format_dev(dev, r.n, 1 + nm.max_name + 1 + D + 1 + D + 3 + r.k + 1, call, sink)
    finally:
        nm.free()


def host_format() -> bool:
    """KMAN_HOST_FORMAT=1: format on host threads (kman_format_*) from
    downloaded results instead of on the device."""
    return os.environ.get("KMAN_HOST_FORMAT", "0") not in ("", "0")


def _to(sink, data):
    if sink is None:
        return data
    sink.write(data)
    return None


def emit_count(dev: Device, r: CountResult, sink=None):
    """The count output text of a device-resident result: returned, or
    written to the binary file `sink`."""
    if host_format():
        ukeys, counts = download_count(dev, r)
        return _to(sink, format_count(ukeys, counts, r.k))
    return format_count_dev(dev, r, sink)


def emit_uniq(p: Parsed, r: UniqResult, sink=None):
    """The uniq output text of a device-resident result over one input."""
    if host_format():
        keys, pos = download_uniq(p.dev, r)
        return _to(sink, format_fasta(keys, pos, r.k, p))
    return format_uniq_dev(p, r, sink)


def download_count(dev: Device, r: CountResult):
    ukeys = dev.download(r.ukeys, r.n, np.uint64)
    counts = dev.download(r.counts, r.n, np.uint32 if r.count_bytes == 4 else np.uint64)
    return ukeys, counts


def download_uniq(dev: Device, r: UniqResult):
    keys = dev.download(r.keys, r.n, np.uint64)
    pos = dev.download(r.pos, r.n, np.uint32 if r.pos_bytes == 4 else np.uint64)
    return keys, pos


# ------------------------------------------------------------------ pipelines


_CODE_TABLE = np.full(128, 4, dtype=np.uint8)
for _i, _c in enumerate("ACGT"):
    _CODE_TABLE[ord(_c)] = _i
    _CODE_TABLE[ord(_c.lower())] = _i


def decode_key(key: int, k: int) -> str:
    """2-bit MSB-first key -> upper-case sequence."""
    return "".join("ACGT"[(int(key) >> (2 * (k - 1 - j))) & 3] for j in range(k))


def kmers_of_sequence(seq: str, k: int, rc: bool, dev: Optional[Device] = None):
    """Keys + pos payloads of every valid window of one sequence string
    (Sequence.yield_kmers, seq.py:285-328), enumerated by kman_extract."""
    _check_k(k)
    dev = dev or default_device()
    cp = np.frombuffer(seq.encode("utf-32-le"), dtype=np.uint32)
    codes = np.where(cp < 128, _CODE_TABLE[np.minimum(cp, 127)], 4).astype(np.uint8)
    n = len(codes)
    if n < k:
        return np.zeros(0, np.uint64), np.zeros(0, np.uint64)
    codes[0] |= 8
    buf = dev.alloc(n + 64)
    try:
        dev.upload(buf, np.concatenate([codes, np.full(64, 4, np.uint8)]))
        p = Parsed(dev, buf, n, 1, np.zeros(1, np.uint64), np.zeros(1, np.uint64), [b""], b"",
                   np.zeros(2, np.uint64))
        km = extract(p, k, rc, want_pos=True)
        try:
            keys = dev.download(km.keys, km.n, np.uint64)
            pos = dev.download(km.pos, km.n, np.uint32 if km.pos_bytes == 4 else np.uint64).astype(np.uint64)
        finally:
            km.free()
    finally:
        buf.free()
    return keys, pos


def read_input(path: str) -> bytes:
    """Bytes of a FASTA file; ``.gz`` is decompressed (batcher.py:480)."""
    if path.endswith(".gz"):
        import gzip

        with gzip.open(path, "rb") as fh:
            text = fh.read()
    else:
        with open(path, "rb") as fh:
            text = fh.read()
    phases.mark("file_read")
    return text


def count_groups(p: Parsed, k: int, rc: bool = False, canonical: bool = False, ordered: bool = True) -> CountResult:
    """(key, count) per distinct k-mer on the device: the region path, else
    the prefix-split path (None only when there are no k-mers).
    ordered=False: the rows may come in any order (a spectrum needs only
    the multiset; the key rounds then skip merging a redone key range).
    k > 32: a WordsResult (word keys, its counts in .vals)."""
    if k > MAX_K:
        return words_groups(p, k, rc, "count", canonical)
    # a spectrum (ordered=False) of canonical keys counts mixed keys
    # (KMAN_MIXED): the same counts, uniform buckets for the region passes
    mixed = canonical and not ordered
    r = groups(p, k, rc, "count", canonical, mixed)
    if r is not None:
        return r
    if p.n_bases:
        from . import dist

        r = dist.local_groups(p, k, rc, "count", canonical, ordered=ordered)
        if r is not None:
            return r
    km = extract_sorted(p, k, rc, want_pos=False, canonical=canonical)
    try:
        if km.n == 0:
            return None
        return rle_count(km, p.dev)
    finally:
        km.free()


def abundance_hist(text: bytes, k: int, canonical: bool = True, nbins: int = 10001,
                   dev: Optional[Device] = None) -> np.ndarray:
    """k-mer abundance spectrum (BASELINE config 5; SURVEY §8f-1, not in the
    reference): h[c] = distinct (canonical) k-mers seen c times, h[-1] every
    count >= nbins - 1 (kman_count_hist over the count output)."""
    dev = dev or default_device()
    _check_k(k, wide=True)
    p = parse(dev, text)
    try:
        r = count_groups(p, k, False, canonical, ordered=False)
        d_h = dev.alloc(8 * nbins)
        try:
            if r is None:
                return np.zeros(nbins, np.uint64)
            try:
                cnt, cb = (r.vals, r.val_bytes) if isinstance(r, WordsResult) else (r.counts, r.count_bytes)
                N.check(dev.ctx, N.lib().kman_count_hist(dev.ctx, c_void_p(cnt.ptr), cb, r.n,
                                                         c_void_p(d_h.ptr), nbins), "kman_count_hist")
                return dev.download(d_h, nbins, np.uint64)
            finally:
                free_result(r)
        finally:
            d_h.free()
    finally:
        p.free()


def format_hist(h: np.ndarray) -> bytes:
    """``"%d\t%d\n" % (count, n_kmers)`` for every non-empty bin; the last bin
    reads ``">=N"``."""
    out = []
    last = len(h) - 1
    for c in np.nonzero(h)[0].tolist():
        out.append("%s\t%d\n" % ((">=%d" % c) if c == last else str(c), int(h[c])))
    return "".join(out).encode()


def _fits(p: Parsed, k: int, rc: bool, mode: str) -> bool:
    """Does the single-batch general path (extract_sorted + rle_*) fit the
    free HBM?  If not, the multi-batch join (ranged_groups) takes the input."""
    n = p.n_bases * (2 if rc else 1)
    pb = 4 if 2 * p.n_bases <= 0xFFFFFFFF else 8
    need = n * (16 + 8 + (3 * pb if mode == "uniq" else (4 if n <= 0xFFFFFFFF else 8)))
    return need <= 0.85 * mem_info(p.dev)[0]


def nwords(k: int) -> int:
    """64-bit words per k-mer of the any-k path (words.hip): ceil(k / 32)."""
    return (k + 31) // 32


@dataclass
class Words:
    """k-mer keys of any k as W word planes (words.hip layout: word 0 the
    first k - 32 (W - 1) bases, then 32 bases per word, all MSB-first; word j
    of item i at words[j * stride + i]) + an optional u64 pos payload."""

    words: DeviceBuffer
    pos: Optional[DeviceBuffer]
    n: int
    k: int
    stride: int

    @property
    def W(self) -> int:
        return nwords(self.k)

    def plane(self, j: int) -> int:
        return self.words.ptr + 8 * j * self.stride

    def free(self) -> None:
        for b in (self.words, self.pos):
            if b is not None:
                b.free()


@dataclass
class WordsResult:
    """count / uniq rows of k > 32: keys as W word planes (stride n)."""

    words: DeviceBuffer
    vals: DeviceBuffer
    val_bytes: int
    n: int
    k: int
    mode: str

    @property
    def W(self) -> int:
        return nwords(self.k)

    def free(self) -> None:
        self.words.free()
        self.vals.free()


def extract_words(p: Parsed, k: int, rc: bool, want_pos: bool, canonical: bool = False) -> Words:
    """Keys (+ u64 pos) of the stream as word planes, in stream order
    (Sequence.yield_kmers, seq.py:285-328): kman_extract_wide's rolled
    LDS-staged kernel for k <= 64 (its (hi, lo) are planes 0 and 1),
    kman_extract_words beyond."""
    _check_k(k, wide=True)
    dev, L = p.dev, N.lib()
    n = count_kmers(p, k, rc, canonical)
    W = nwords(k)
    words = dev.alloc(8 * W * max(n, 1))
    pos = dev.alloc(8 * max(n, 1)) if want_pos else None
    w = Words(words, pos, n, k, max(n, 1))
    if n == 0:
        return w
    got = c_uint64(0)
    try:
        if k <= MAX_K_WIDE:
            N.check(dev.ctx, L.kman_extract_wide(dev.ctx, c_void_p(p.codes.ptr), p.n_bases, k,
                                                 flags_for(rc, want_pos, canonical), c_void_p(w.plane(0)),
                                                 c_void_p(w.plane(1)), c_void_p(pos.ptr) if pos else None, 8, n,
                                                 byref(got)), "kman_extract_wide")
        else:
            N.check(dev.ctx, L.kman_extract_words(dev.ctx, c_void_p(p.codes.ptr), p.n_bases, k,
                                                  flags_for(rc, want_pos, canonical), c_void_p(words.ptr), w.stride,
                                                  c_void_p(pos.ptr) if pos else None, 8, n, byref(got)),
                    "kman_extract_words")
    except BaseException:
        w.free()
        raise
    assert int(got.value) == n
    return w


def sort_words(w: Words, start: int = 0, per_batch: Optional[int] = None, dev: Optional[Device] = None) -> Words:
    """A stably sorted copy of word keys (+ pos): LSD over the planes, last
    word first, each a stable kman_sort of the gathered plane carrying the
    permutation (ties keep stream order, as the reference's Timsort,
    batch.py:156-168); per_batch: items in consecutive chunks of that many
    from stream index `start` sorted chunk by chunk (one Batch each) -- a
    final stable sort by the chunk tag (kman_batch_tags)."""
    dev, L = dev or w.words.dev, N.lib()
    n, W, k = w.n, w.W, w.k
    out = Words(dev.alloc(8 * W * max(n, 1)), dev.alloc(8 * max(n, 1)) if w.pos is not None else None, n, k,
                max(n, 1))
    if n == 0:
        return out
    bufs = [dev.alloc(8 * n) for _ in range(4)]
    try:
        perm, key, alt_k, alt_p = bufs
        N.check(dev.ctx, L.kman_iota_u64(dev.ctx, c_void_p(perm.ptr), n), "iota")
        res = c_int(0)

        def stable(keys_, bits):
            nonlocal perm, alt_k, alt_p
            N.check(dev.ctx, L.kman_sort(dev.ctx, c_void_p(keys_.ptr), c_void_p(alt_k.ptr), c_void_p(perm.ptr),
                                         c_void_p(alt_p.ptr), 8, n, bits, None, byref(res)), "kman_sort")
            if res.value:  # (the sorted copy is in the alternates)
                perm, alt_p = alt_p, perm
                return alt_k, keys_
            return keys_, alt_k

        h = k - 32 * (W - 1)
        for j in reversed(range(W)):
            N.check(dev.ctx, L.kman_gather(dev.ctx, c_void_p(w.plane(j)), c_void_p(perm.ptr), n, c_void_p(key.ptr), 8),
                    "gather")
            key, alt_k = stable(key, 64 if j else 2 * h)
        if per_batch is not None:
            last = (start + n - 1) // per_batch
            N.check(dev.ctx, L.kman_batch_tags(dev.ctx, c_void_p(perm.ptr), n, start, per_batch, c_void_p(key.ptr)),
                    "kman_batch_tags")
            key, alt_k = stable(key, max(1, int(last).bit_length()))
        for j in range(W):
            N.check(dev.ctx, L.kman_gather(dev.ctx, c_void_p(w.plane(j)), c_void_p(perm.ptr), n,
                                           c_void_p(out.plane(j)), 8), "gather")
        if w.pos is not None:
            N.check(dev.ctx, L.kman_gather(dev.ctx, c_void_p(w.pos.ptr), c_void_p(perm.ptr), n, c_void_p(out.pos.ptr),
                                           8), "gather")
    except BaseException:
        out.free()
        raise
    finally:
        for b in bufs:
            b.free()
    return out


def rle_words(w: Words, mode: str) -> WordsResult:
    """Run-length rows of sorted word keys (Crawler.do_batch + the count /
    uniq writers, join.py:95-130, 244-285)."""
    dev, L = w.words.dev, N.lib()
    n, W = w.n, w.W
    uniq = mode == "uniq"
    vb = 8 if uniq else (4 if n <= 0xFFFFFFFF else 8)
    ow = dev.alloc(8 * W * max(n, 1))
    ov = dev.alloc(vb * max(n, 1))
    out = c_uint64(0)
    try:
        N.check(dev.ctx, L.kman_rle_words(dev.ctx, N.KMAN_FINISH_UNIQ if uniq else N.KMAN_FINISH_COUNT,
                                          c_void_p(w.words.ptr), W, w.stride, c_void_p(w.pos.ptr) if uniq else None,
                                          8, n, c_void_p(ow.ptr), max(n, 1), c_void_p(ov.ptr), vb, byref(out)),
                "kman_rle_words")
    except BaseException:
        ow.free()
        ov.free()
        raise
    # (planes keep the input's stride n: row j's word q at ow[q * n + j])
    return WordsResult(ow, ov, vb, int(out.value), w.k, mode)


def words_groups(p: Parsed, k: int, rc: bool, mode: str, canonical: bool = False) -> Optional[WordsResult]:
    """k > 32 (seq.py:285-328 has no k limit): the keys as word planes
    (extract_words), an LSD sort over the planes (sort_words,
    batch.py:156-168), kman_rle_words (join.py:95-130, 244-285).  None when
    the stream has no k-mers."""
    w = extract_words(p, k, rc, mode == "uniq", canonical)
    try:
        if w.n == 0:
            return None
        sw = sort_words(w)
    finally:
        w.free()
    try:
        return rle_words(sw, mode)
    finally:
        sw.free()


wide_groups = words_groups  # (the word-pair name of round 2: k in 33..64 is W = 2)


def download_words(dev: Device, words: DeviceBuffer, n: int, k: int, stride: Optional[int] = None) -> np.ndarray:
    """Word planes to a host (n, W) uint64 array."""
    W = nwords(k)
    stride = n if stride is None else stride
    flat = dev.download(words, W * stride, np.uint64) if n else np.zeros(0, np.uint64)
    return np.ascontiguousarray(flat.reshape(W, stride)[:, :n].T) if n else np.zeros((0, W), np.uint64)


def decode_words(row, k: int) -> str:
    """The k-mer text of one (W,) word row."""
    W = nwords(k)
    h = k - 32 * (W - 1)
    return "".join(decode_key(int(x), h if j == 0 else 32) for j, x in enumerate(row))


def join_groups(p: Parsed, k: int, rc: bool, mode: str, max_keys: Optional[int] = None):
    """The count / uniq result of the whole stream of p on the device, by the
    fastest path that takes it: the region path (kman_groups); the multi-batch
    join (RangedJoin) when the single-batch general path does not fit the
    free HBM or max_keys asks for it; else the general path (extract_sorted +
    rle_*); k > 32: the word-pair path (wide_groups).  None when the stream
    has no k-mers."""
    if k > MAX_K:
        return words_groups(p, k, rc, mode)
    r = groups(p, k, rc, mode) if max_keys is None else None
    if r is None and max_keys is None and p.n_bases:
        # outside kman_groups (too many k-mers for its regions, -r on large
        # inputs, skewed keys): the key rounds of the multi-GPU path on one GPU
        from . import dist

        r = dist.local_groups(p, k, rc, mode)
    if r is None and (max_keys is not None or not _fits(p, k, rc, mode)):
        r = ranged_groups(p, k, rc, mode, max_keys)
    if r is None:
        km = extract_sorted(p, k, rc, want_pos=mode == "uniq")
        try:
            if km.n == 0:
                return None
            r = rle_count(km, p.dev) if mode == "count" else rle_uniq(km, p.dev)
        finally:
            km.free()
    return r


def free_result(r) -> None:
    if r is None:
        return
    if isinstance(r, WordsResult):
        bs = (r.words, r.vals)
    else:
        bs = (r.ukeys, r.counts) if isinstance(r, CountResult) else (r.keys, r.pos)
    for b in bs:
        b.free()


def _emit_words(p: Parsed, r: WordsResult, sink=None):
    """Word-key rows as the reference's text: built on the device
    (kman_format_*_words_dev), or by the host writers (kman_format_*_words)
    with KMAN_HOST_FORMAT=1."""
    dev, L = p.dev, N.lib()
    vb = r.val_bytes
    # (row j's word q at words[q * n + j]: a slice of rows is the same planes offset by i0)
    if not host_format():
        if r.mode == "count":
            def call(i0, m, d_out, cap, used):
                return L.kman_format_count_words_dev(dev.ctx, c_void_p(r.words.ptr + 8 * i0), max(r.n, 1),
                                                     c_void_p(r.vals.ptr + vb * i0), vb, m, r.k, d_out, cap,
                                                     byref(used))

            return _format_dev(dev, r.n, r.k + 2 + 20, call, sink)
        nm = DeviceNames(p)
        try:
            D = len(str(p.n_bases + r.k))

            def call(i0, m, d_out, cap, used):
                return L.kman_format_uniq_words_dev(dev.ctx, c_void_p(r.words.ptr + 8 * i0), max(r.n, 1),
                                                    c_void_p(r.vals.ptr + vb * i0), vb, m, r.k,
                                                    c_void_p(nm.names.ptr), c_void_p(nm.off.ptr), c_void_p(nm.rec.ptr),
                                                    nm.n_records, d_out, cap, byref(used))

            return _format_dev(dev, r.n, 1 + nm.max_name + 1 + D + 1 + D + 3 + r.k + 1, call, sink)
        finally:
            nm.free()
    words = dev.download(r.words, r.W * max(r.n, 1), np.uint64)
    vals = dev.download(r.vals, r.n, np.uint32 if vb == 4 else np.uint64)
    if r.mode == "count":
        return _to(sink, _format(L.kman_format_count_words, words.ctypes.data_as(c_void_p), max(r.n, 1),
                                 vals.ctypes.data_as(c_void_p), vb, r.n, r.k))
    names = ctypes.create_string_buffer(p.names_blob, max(1, len(p.names_blob)))
    off = np.ascontiguousarray(p.name_off, dtype=np.uint64)
    rs = np.ascontiguousarray(p.rec_seq, dtype=np.uint64)
    return _to(sink, _format(L.kman_format_uniq_words, words.ctypes.data_as(c_void_p), max(r.n, 1),
                             vals.ctypes.data_as(c_void_p), vb, r.n, r.k, names, off.ctypes.data_as(c_void_p),
                             rs.ctypes.data_as(c_void_p), p.n_records))


_emit_wide = _emit_words  # (round-2 name)


def count_text(text: bytes, k: int, rc: bool = False, dev: Optional[Device] = None,
               max_keys: Optional[int] = None) -> bytes:
    """``kmer count`` output bytes for a FASTA text (SEQ_COUNT mode).
    max_keys: run the multi-batch join with key ranges of at most that many
    k-mers (by default only when the single batch does not fit the HBM)."""
    dev = dev or default_device()
    _check_k(k, wide=True)
    p = parse(dev, text)
    try:
        check_empty_names(p, k)
        r = join_groups(p, k, rc, "count", max_keys)
        if r is None:
            return b""
        try:
            if isinstance(r, WordsResult):
                return _emit_words(p, r)
            return emit_count(dev, r)
        finally:
            free_result(r)
    finally:
        p.free()


def uniq_text(text: bytes, k: int, rc: bool = False, dev: Optional[Device] = None,
              max_keys: Optional[int] = None) -> bytes:
    """``kmer uniq`` output bytes for a FASTA text (UNIQUE mode); max_keys as
    in count_text."""
    dev = dev or default_device()
    _check_k(k, wide=True)
    p = parse(dev, text)
    try:
        check_empty_names(p, k)
        r = join_groups(p, k, rc, "uniq", max_keys)
        if r is None:
            return b""
        try:
            if isinstance(r, WordsResult):
                return _emit_words(p, r)
            return emit_uniq(p, r)
        finally:
            free_result(r)
    finally:
        p.free()


# ------------------------------------------------------- resident pipeline


class ResidentPipeline:
    """One FASTA text resident in HBM, every buffer preallocated: ``step()``
    runs parse -> extract -> sort -> count|uniq with no allocation, leaving
    the result device-resident (what bench.py times)."""

    def __init__(self, dev: Device, text: bytes, k: int, mode: str = "uniq", rc: bool = False,
                 pos_bytes: Optional[int] = None, path: str = "region"):
        _check_k(k)
        if mode not in ("count", "uniq"):
            raise ValueError(mode)
        if path not in ("region", "split", "full"):
            raise ValueError(path)
        # region: kman_groups (default; falls back to split when the input is
        # outside the region path); split: prefix passes + kman_finish; full:
        # every bit in global passes + kman_rle_* (kept for A/B runs)
        self.path = path
        self.work = None
        self.dev, self.k, self.mode, self.rc = dev, k, mode, rc
        n = len(text)
        self.n_bytes = n
        self.text = dev.alloc(n + 64)
        dev.upload(self.text, text)
        self.codes = dev.alloc(n + 64)
        self.rec_cap = n // 2 + 1
        self.rec_hdr = dev.alloc(8 * self.rec_cap)
        self.rec_seq = dev.alloc(8 * self.rec_cap)
        self.bound = max(1, n * (2 if rc else 1))
        self.pos_bytes = pos_bytes or (4 if 2 * n <= 0xFFFFFFFF else 8)
        want_pos = mode == "uniq"
        self.keys = dev.alloc(8 * self.bound)
        self.alt = dev.alloc(8 * self.bound)
        self.pos = dev.alloc(self.pos_bytes * self.bound) if want_pos else None
        self.pos_alt = dev.alloc(self.pos_bytes * self.bound) if want_pos else None
        self.hist = dev.alloc(8 * 256 * 8)
        self.out_keys = dev.alloc(8 * self.bound)
        self.count_bytes = 4 if self.bound <= 0xFFFFFFFF else 8
        self.out_vals = dev.alloc((self.pos_bytes if want_pos else self.count_bytes) * self.bound)
        self.lo_bit = split_bits(self.bound, 2 * k) if path == "split" else 0
        self.flags = flags_for(rc, want_pos) | N.KMAN_HIST_LO(self.lo_bit)
        self.n_kmers = 0
        self.n_out = 0
        self.n_bases = 0
        self.sorted_in_alt = False
        if self.path == "region":
            self._parse()
            wb = c_uint64(0)
            m = N.KMAN_FINISH_UNIQ if mode == "uniq" else N.KMAN_FINISH_COUNT
            r = N.lib().kman_groups_plan(self.n_bases, k, flags_for(rc, want_pos), m, byref(wb))
            if r == N.KMAN_EFALLBACK:
                self._to_split()
            else:
                N.check(dev.ctx, r, "kman_groups_plan")
                self.work = dev.alloc(int(wb.value))
                self.work_bytes = int(wb.value)

    def _to_split(self) -> None:
        """Switch to the prefix-split path with its own digit plan (the region
        path plans no prefix passes: lo_bit 0 would run every key bit through
        the global passes)."""
        self.path = "split"
        if self.work is not None:
            self.work.free()
            self.work = None
        self.lo_bit = split_bits(self.bound, 2 * self.k)
        self.flags = flags_for(self.rc, self.mode == "uniq") | N.KMAN_HIST_LO(self.lo_bit)

    def _parse(self) -> None:
        info = N.ParseInfo()
        N.check(self.dev.ctx, N.lib().kman_parse_fasta(self.dev.ctx, c_void_p(self.text.ptr), self.n_bytes,
                                                        c_void_p(self.codes.ptr), c_void_p(self.rec_hdr.ptr),
                                                        c_void_p(self.rec_seq.ptr), self.rec_cap, byref(info)),
                "kman_parse_fasta")
        self.n_bases = int(info.n_bases)

    def extract_only(self) -> int:
        """parse + extract (stream-order keys / pos in self.keys / self.pos)."""
        L, ctx = N.lib(), self.dev.ctx
        info = N.ParseInfo()
        N.check(ctx, L.kman_parse_fasta(ctx, c_void_p(self.text.ptr), self.n_bytes, c_void_p(self.codes.ptr),
                                        c_void_p(self.rec_hdr.ptr), c_void_p(self.rec_seq.ptr), self.rec_cap,
                                        byref(info)), "kman_parse_fasta")
        self.n_bases = int(info.n_bases)
        n = c_uint64(0)
        pos = c_void_p(self.pos.ptr) if self.pos else c_void_p(None)
        N.check(ctx, L.kman_extract(ctx, c_void_p(self.codes.ptr), self.n_bases, self.k, self.flags,
                                    c_void_p(self.keys.ptr), pos, self.pos_bytes, self.bound, None, byref(n)),
                "kman_extract")
        self.n_kmers = int(n.value)
        return self.n_kmers

    def step(self) -> int:
        L, ctx = N.lib(), self.dev.ctx
        self._parse()
        if self.path == "region":
            m = N.KMAN_FINISH_UNIQ if self.mode == "uniq" else N.KMAN_FINISH_COUNT
            ob = self.count_bytes if self.mode == "count" else self.pos_bytes
            nk, no = c_uint64(0), c_uint64(0)
            r = L.kman_groups(ctx, c_void_p(self.codes.ptr), self.n_bases, self.k, self.flags & 0xff, m,
                              c_void_p(self.work.ptr), self.work_bytes, c_void_p(self.out_keys.ptr),
                              c_void_p(self.out_vals.ptr), ob, byref(nk), byref(no))
            if r != N.KMAN_EFALLBACK:
                N.check(ctx, r, "kman_groups")
                self.n_kmers, self.n_out = int(nk.value), int(no.value)
                return self.n_kmers
            # a region overflowed (skewed input): the general path from here on
            self._to_split()
        n = c_uint64(0)
        res = c_int(0)
        pos = c_void_p(self.pos.ptr) if self.pos else c_void_p(None)
        vb = self.pos_bytes if self.pos else 0
        pos_alt = c_void_p(self.pos_alt.ptr if self.pos_alt else None)
        if self.path == "split":
            # extraction fused with the first prefix pass, then the other prefix passes
            N.check(ctx, L.kman_extract_sorted(ctx, c_void_p(self.codes.ptr), self.n_bases, self.k,
                                               self.flags & 0xff, self.lo_bit, c_void_p(self.keys.ptr),
                                               c_void_p(self.alt.ptr), pos, pos_alt, self.pos_bytes, self.bound,
                                               byref(n), byref(res)), "kman_extract_sorted")
            self.n_kmers = int(n.value)
        else:
            N.check(ctx, L.kman_memset(ctx, c_void_p(self.hist.ptr), 0, 8 * 256 * 8), "memset")
            N.check(ctx, L.kman_extract(ctx, c_void_p(self.codes.ptr), self.n_bases, self.k, self.flags,
                                        c_void_p(self.keys.ptr), pos, self.pos_bytes, self.bound,
                                        c_void_p(self.hist.ptr), byref(n)), "kman_extract")
            self.n_kmers = int(n.value)
            N.check(ctx, L.kman_sort(ctx, c_void_p(self.keys.ptr), c_void_p(self.alt.ptr), pos, pos_alt, vb,
                                     self.n_kmers, 2 * self.k, c_void_p(self.hist.ptr), byref(res)), "kman_sort")
        self.sorted_in_alt = bool(res.value)
        skeys = self.alt if res.value else self.keys
        out = c_uint64(0)
        if self.path == "split":
            spos = self.pos_alt if res.value else self.pos
            other = self.keys if res.value else self.alt
            opos = self.pos if res.value else self.pos_alt
            mode = N.KMAN_FINISH_COUNT if self.mode == "count" else N.KMAN_FINISH_UNIQ
            ob = self.count_bytes if self.mode == "count" else self.pos_bytes
            N.check(ctx, L.kman_finish(ctx, c_void_p(skeys.ptr), c_void_p(other.ptr),
                                       c_void_p(spos.ptr if spos else None), c_void_p(opos.ptr if opos else None), vb,
                                       self.n_kmers, 2 * self.k, self.lo_bit, mode, c_void_p(self.out_keys.ptr),
                                       c_void_p(self.out_vals.ptr), ob, byref(out)), "kman_finish")
        elif self.mode == "count":
            N.check(ctx, L.kman_rle_count(ctx, c_void_p(skeys.ptr), self.n_kmers, c_void_p(self.out_keys.ptr),
                                          c_void_p(self.out_vals.ptr), self.count_bytes, byref(out)),
                    "kman_rle_count")
        else:
            spos = self.pos_alt if res.value else self.pos
            N.check(ctx, L.kman_rle_uniq(ctx, c_void_p(skeys.ptr), c_void_p(spos.ptr), self.pos_bytes,
                                         self.n_kmers, c_void_p(self.out_keys.ptr), c_void_p(self.out_vals.ptr),
                                         byref(out)), "kman_rle_uniq")
        self.n_out = int(out.value)
        return self.n_kmers

    @property
    def n_sorted(self) -> int:
        return self.n_kmers

    def timing(self, enable: bool) -> None:
        N.check(self.dev.ctx, N.lib().kman_timing_enable(self.dev.ctx, 1 if enable else 0), "timing")

    def timed(self, tag: str):
        n, ms = c_uint64(0), ctypes.c_double(0)
        N.check(self.dev.ctx, N.lib().kman_timing_query(self.dev.ctx, tag.encode(), byref(n), byref(ms)), "timing")
        return int(n.value), float(ms.value)

    def free(self) -> None:
        for b in (self.text, self.codes, self.rec_hdr, self.rec_seq, self.keys, self.alt, self.pos, self.pos_alt,
                  self.hist, self.out_keys, self.out_vals, self.work):
            if b is not None:
                b.free()
