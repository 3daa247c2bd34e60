"""Byte-range shards of ONE FASTA, loaded onto the device in chunks.

SURVEY §8e: rank q of G takes the bytes [start_q, start_{q+1}) of the file,
cut at line starts, plus a halo of the k-1 bases that follow (up to the next
header line): a window belongs to the shard that holds its first base, so
the windows of all shards are exactly the windows of the whole file
(Sequence.yield_kmers over every record, kmermaid/seq.py:285-328;
FastaBatcher's one stream over all records, kmermaid/batcher.py:386-392).

The same cut serves the streamed upload of one input (``ShardCodes`` with
chunk_bytes): chunks at line starts are copied host -> device on the
context's copy stream while the previous chunk is parsed
(kman_parse_fasta_at, a chunk inside a record starts in the sequence-line
state), so a step that starts from host bytes does not pay the whole H2D copy
before the first kernel.

A reader is any object with ``size`` and ``read(lo, hi) -> bytes``; it may
also offer ``ptr(lo)`` (a pinned host address of byte lo: async copies) or
``gen(dev, buf, lo, hi)`` (writes the bytes straight into a device buffer:
the benchmark's synthetic file, kman_synth_fasta).
"""

from __future__ import annotations

import ctypes
from ctypes import byref, c_void_p
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import _native as N
from . import engine

LF, CR, GT = 0x0A, 0x0D, 0x3E
_WS = b" \t\n\r\x0b\x0c\x1c\x1d\x1e\x1f"
_SCAN = 1 << 16


class BytesReader:
    """A reader over an in-memory bytes-like object (tests, small inputs)."""

    def __init__(self, data):
        self.data = memoryview(data).cast("B")
        self.size = len(self.data)

    def read(self, lo: int, hi: int) -> bytes:
        return bytes(self.data[max(0, lo):max(0, min(hi, self.size))])


class PinnedReader(BytesReader):
    """Bytes held in pinned host memory (kman_host_alloc): chunk uploads are
    asynchronous and overlap the parse of the previous chunk."""

    def __init__(self, dev: engine.Device, data=None, size: Optional[int] = None):
        n = len(data) if data is not None else int(size)
        hp = c_void_p()
        N.check(dev.ctx, N.lib().kman_host_alloc(dev.ctx, byref(hp), max(1, n)), "kman_host_alloc")
        self.dev, self.addr = dev, hp.value
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * max(1, n)).from_address(self.addr))[:n]
        if data is not None:
            self.array[:] = np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)
        super().__init__(self.array)

    def ptr(self, lo: int) -> int:
        return self.addr + int(lo)

    def free(self) -> None:
        if self.addr:
            N.lib().kman_host_free(self.dev.ctx, c_void_p(self.addr))
            self.addr = None


class SynthReader:
    """The benchmark's global synthetic FASTA (tests/golden/inputs.py
    SynthLayout): host reads by the numpy restatement, device chunks by
    kman_synth_fasta."""

    def __init__(self, layout):
        self.lay = layout
        self.size = layout.size

    def read(self, lo: int, hi: int) -> bytes:
        return self.lay.read(lo, hi)

    def gen(self, dev: engine.Device, buf: engine.DeviceBuffer, lo: int, hi: int) -> None:
        tab = np.ascontiguousarray(self.lay.tab, dtype=np.uint64)
        N.check(dev.ctx, N.lib().kman_synth_fasta(dev.ctx, c_void_p(buf.ptr), lo, hi - lo, self.lay.seed,
                                                  tab.ctypes.data_as(c_void_p), self.lay.n_records, self.lay.width),
                "kman_synth_fasta")


# ---------------------------------------------------------------- host cuts


def line_start_at_or_after(rd, pos: int) -> int:
    """First line start >= pos (universal newlines: after LF, after CR not
    followed by LF); rd.size when there is none."""
    size = rd.size
    if pos <= 0:
        return 0
    if pos >= size:
        return size
    two = rd.read(pos - 1, pos + 1)
    if two[0] == LF or (two[0] == CR and two[1] != LF):
        return pos
    at = pos
    while at < size:
        blk = rd.read(at, min(size, at + _SCAN))
        i, j = blk.find(b"\n"), blk.find(b"\r")
        hits = [x for x in (i, j) if x >= 0]
        if hits:
            t = at + min(hits)
            if blk[min(hits)] == CR:
                return t + 2 if rd.read(t + 1, t + 2) == b"\n" else t + 1
            return t + 1
        at += len(blk)
    return size


def first_header(rd) -> int:
    """Byte offset of the first line that starts with '>' (parsers.py:43-56:
    everything before it is skipped); rd.size when there is none."""
    pos = 0
    while pos < rd.size:
        if rd.read(pos, pos + 1) == b">":
            return pos
        pos = line_start_at_or_after(rd, pos + 1)
    return rd.size


def halo_end(rd, own_end: int, k: int) -> int:
    """End of the halo after a shard: whole lines after own_end until they
    hold k-1 non-whitespace bytes (at least k-1 bases), a header line, or EOF.
    The halo's bases past the first k-1 are cut off after parsing."""
    need, pos = k - 1, own_end
    while need > 0 and pos < rd.size:
        if rd.read(pos, pos + 1) == b">":
            break
        nxt = line_start_at_or_after(rd, pos + 1)
        need -= len(rd.read(pos, nxt).translate(None, _WS))
        pos = nxt
    return pos


@dataclass
class ShardSpec:
    rank: int
    start: int      # first byte (a line start)
    own_end: int    # first byte of the next shard
    halo_end: int   # end of the halo lines
    h0: int         # first header line of the file


def shard_specs(rd, world: int, k: int) -> List[ShardSpec]:
    """The G byte ranges of one FASTA: cuts at the line starts at or after
    q * size / G (a one-line record cannot be cut: its shard takes it whole and
    the next shards start after it)."""
    h0 = first_header(rd)
    if h0 >= rd.size:
        raise AssertionError("premature end of file or empty file")  # parsers.py:105-107
    cuts = [0]
    for q in range(1, world):
        cuts.append(max(cuts[-1], line_start_at_or_after(rd, q * rd.size // world)))
    cuts.append(rd.size)
    out = []
    for q in range(world):
        s, e = cuts[q], cuts[q + 1]
        h = halo_end(rd, e, k) if h0 < e < rd.size else e
        out.append(ShardSpec(q, s, e, h, h0))
    return out


def chunk_cuts(rd, lo: int, hi: int, chunk: int) -> List[int]:
    """Line-start cuts of [lo, hi) into pieces of about `chunk` bytes."""
    cuts = [lo]
    while cuts[-1] < hi:
        nxt = line_start_at_or_after(rd, cuts[-1] + chunk) if cuts[-1] + chunk < hi else hi
        cuts.append(min(max(nxt, cuts[-1] + 1), hi))
    return cuts


# ------------------------------------------------------------ device shard


def _name_at(rd, hdr: int) -> bytes:
    """Record name of the header line at byte hdr (batcher.py:551)."""
    n = 256
    while True:
        line = rd.read(hdr, hdr + n)
        cut = [x for x in (line.find(b"\n"), line.find(b"\r")) if x >= 0]
        if cut or hdr + n >= rd.size:
            return engine._title_name(line[:min(cut)] if cut else line, 0)
        n *= 4


@dataclass
class ShardCodes:
    """One shard's base codes on the device: n_own bases of its own bytes,
    then at most k-1 halo bases (n_eff in all), then 64 pad codes (4), and
    the records that start in the shard (names, first base index)."""

    dev: engine.Device
    spec: ShardSpec
    k: int
    codes: Optional[engine.DeviceBuffer] = None
    n_own: int = 0
    n_eff: int = 0
    names: List[bytes] = field(default_factory=list)
    rec_seq: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint64))
    timing: dict = field(default_factory=dict)

    def free(self) -> None:
        if self.codes is not None:
            self.codes.free()
            self.codes = None


class ShardLoader:
    """Uploads and parses a shard chunk by chunk into its codes buffer; the
    text staging buffers (two chunks) stay allocated, so load() can run every
    step (the pinned-host benchmark line)."""

    def __init__(self, dev: engine.Device, rd, spec: ShardSpec, k: int, chunk_bytes: int = 256 << 20,
                 resident: bool = False):
        """resident: a shard of one chunk keeps its staged text (and halo) in
        HBM, so every load() after the first only parses (the multi-GPU
        benchmark step then covers the parse like the single-GPU step)."""
        self.dev, self.rd, self.spec, self.k = dev, rd, spec, k
        self.resident, self._staged = resident, False
        own = spec.own_end - spec.start
        self.cuts = chunk_cuts(rd, spec.start, spec.own_end, chunk_bytes)
        big = max([b - a for a, b in zip(self.cuts, self.cuts[1:])] + [spec.halo_end - spec.own_end, 1])
        self.text = [dev.alloc(big + 64), dev.alloc(big + 64)]
        self.rec_cap = 1 << 16
        self.d_hdr = dev.alloc(8 * self.rec_cap)
        self.d_seq = dev.alloc(8 * self.rec_cap)
        self.shard = ShardCodes(dev, spec, k, codes=dev.alloc(own + (spec.halo_end - spec.own_end) + 128))

    def _stage(self, slot: int, lo: int, hi: int) -> None:
        """Bytes [lo, hi) into text buffer `slot`: generated on the device,
        an async copy from pinned memory, or a synchronous upload."""
        buf = self.text[slot]
        if hi <= lo:
            return
        if hasattr(self.rd, "gen"):
            self.rd.gen(self.dev, buf, lo, hi)
            return
        if hasattr(self.rd, "ptr"):
            N.check(self.dev.ctx, N.lib().kman_copy_h2d_async(self.dev.ctx, c_void_p(buf.ptr), c_void_p(self.rd.ptr(lo)),
                                                             hi - lo, slot), "kman_copy_h2d_async")
            return
        self.dev.upload(buf, self.rd.read(lo, hi))

    def _wait(self, slot: int) -> None:
        if hasattr(self.rd, "ptr") and not hasattr(self.rd, "gen"):
            N.check(self.dev.ctx, N.lib().kman_copy_wait(self.dev.ctx, slot), "kman_copy_wait")

    def _parse(self, slot: int, lo: int, hi: int, code_off: int):
        """Parse chunk [lo, hi) (staged in `slot`) into codes from code_off;
        returns (n_bases, record header offsets, record first bases)."""
        sp = self.spec
        if hi <= lo or hi <= sp.h0:  # empty, or wholly before the first header
            return 0, [], []
        flags = N.KMAN_PARSE_IN_RECORD if lo > sp.h0 else 0
        L, ctx = N.lib(), self.dev.ctx
        while True:
            info = N.ParseInfo()
            rc = L.kman_parse_fasta_at(ctx, c_void_p(self.text[slot].ptr), hi - lo, flags,
                                       c_void_p(self.shard.codes.ptr), code_off, c_void_p(self.d_hdr.ptr),
                                       c_void_p(self.d_seq.ptr), self.rec_cap, byref(info))
            if rc == N.KMAN_ECAP and info.n_records > self.rec_cap:
                self.d_hdr.free()
                self.d_seq.free()
                self.rec_cap = int(info.n_records) + 1024
                self.d_hdr, self.d_seq = self.dev.alloc(8 * self.rec_cap), self.dev.alloc(8 * self.rec_cap)
                continue
            N.check(ctx, rc, "kman_parse_fasta_at")
            break
        R = int(info.n_records)
        hdr = (self.dev.download(self.d_hdr, R, np.uint64) + np.uint64(lo)).tolist() if R else []
        seq = self.dev.download(self.d_seq, R, np.uint64).tolist() if R else []
        return int(info.n_bases), hdr, seq

    def _mark(self, at: int) -> None:
        """Record-start bit on code `at` (a record whose header ended the
        previous chunk: that chunk's parse could not mark a code it did not
        write)."""
        c = self.dev.download(self.shard.codes, 1, np.uint8, offset=at)
        self.dev.upload(self.shard.codes, c | np.uint8(8), offset=at)

    def load(self, on_chunk=None) -> ShardCodes:
        """Upload + parse every chunk (the next chunk's copy behind the
        current parse), then the halo; seal the codes after k-1 halo bases.
        on_chunk(n) runs after each chunk's parse, when the codes below n are
        final (kman_groups_extract queues work behind the next copy)."""
        sh, sp, dev = self.shard, self.spec, self.dev
        n, hdrs, seqs = 0, [], []
        cuts = self.cuts
        pieces = list(zip(cuts, cuts[1:]))
        keep = self.resident and self._staged and len(pieces) <= 1  # the text is still in place
        if pieces and not keep:
            self._stage(0, *pieces[0])
        for i, (lo, hi) in enumerate(pieces):
            slot = i & 1
            if i + 1 < len(pieces):
                if i:  # the parse of chunk i - 1 (slot ^ 1) may still run: the copy must not overwrite its text
                    dev.sync()
                self._stage(slot ^ 1, *pieces[i + 1])
            if not keep:
                self._wait(slot)
            m, h, s = self._parse(slot, lo, hi, n)
            if m and seqs and seqs[-1] == n:
                self._mark(n)  # a record opened at the end of the previous chunk starts here
            n += m
            hdrs += h
            seqs += s
            if on_chunk is not None and i + 1 < len(pieces):
                on_chunk(n)
        sh.n_own = n
        halo = 0
        if sp.halo_end > sp.own_end:
            slot = len(pieces) & 1
            if not keep:
                self._stage(slot, sp.own_end, sp.halo_end)
                self._wait(slot)
            halo, h, _ = self._parse(slot, sp.own_end, sp.halo_end, n)
            assert not h, "a halo holds no header line"
            if halo and seqs and seqs[-1] == n:
                self._mark(n)
        sh.n_eff = n + min(halo, self.k - 1)
        dev.memset(sh.codes, 4, 64, offset=sh.n_eff)
        if sh.names == [] or len(sh.names) != len(hdrs):
            sh.names = [_name_at(self.rd, int(x)) for x in hdrs]
        sh.rec_seq = np.asarray(seqs, dtype=np.uint64)
        dev.sync()
        self._staged = True
        return sh

    def free(self) -> None:
        for b in self.text + [self.d_hdr, self.d_seq]:
            b.free()
        self.shard.free()


def load_text(dev: engine.Device, text: bytes, chunk_bytes: int = 256 << 20) -> engine.Parsed:
    """A whole FASTA text as one shard through the chunked loader: the same
    Parsed as engine.parse (tests compare the two)."""
    rd = BytesReader(text)
    sp = shard_specs(rd, 1, 2)[0]
    ld = ShardLoader(dev, rd, sp, 2, chunk_bytes)
    try:
        sh = ld.load()
        for b in ld.text + [ld.d_hdr, ld.d_seq]:
            b.free()
        names = sh.names
        R = len(names)
        name_off = np.zeros(R + 1, dtype=np.uint64)
        if R:
            name_off[1:] = np.cumsum([len(x) for x in names], dtype=np.uint64)
        return engine.Parsed(dev, sh.codes, sh.n_own, R, np.zeros(R, np.uint64), sh.rec_seq, names, b"".join(names),
                             name_off)
    except BaseException:
        ld.free()
        raise


class StreamedPipeline:
    """``kmer count|uniq`` of a FASTA held in (pinned) host memory, as the
    reference's CLI runs it from its input bytes: every step uploads the text
    in chunks -- each chunk's copy on the copy stream behind the parse and
    (overlap) the region path's first pass over the previous one -- and
    finishes the region path (kman_groups) on the codes, leaving the result
    device-resident (bench.py's pinned-host line)."""

    def __init__(self, dev: engine.Device, reader, k: int, mode: str = "uniq", chunk_bytes: int = 128 << 20,
                 overlap: bool = True):
        self.dev, self.k, self.mode, self.overlap = dev, k, mode, overlap
        self.loader = ShardLoader(dev, reader, shard_specs(reader, 1, k)[0], k, chunk_bytes)
        sh = self.loader.load()
        self.n_bases = sh.n_own
        self.m = N.KMAN_FINISH_UNIQ if mode == "uniq" else N.KMAN_FINISH_COUNT
        self.flags = engine.flags_for(False, mode == "uniq")
        wb = ctypes.c_uint64(0)
        N.check(dev.ctx, N.lib().kman_groups_plan(sh.n_own, k, self.flags, self.m, byref(wb)), "kman_groups_plan")
        self.work_bytes = int(wb.value)
        self.work = dev.alloc(self.work_bytes)
        self.vb = 4
        self.out_keys = dev.alloc(8 * max(1, sh.n_own))
        self.out_vals = dev.alloc(4 * max(1, sh.n_own))
        self.n_kmers = self.n_out = 0

    def step(self) -> int:
        """One pass from the host bytes: with `overlap`, kman_groups' first
        pass runs chunk by chunk (kman_groups_begin / _extract / _end) behind
        the copies of the following chunks; else kman_groups after the load."""
        L, ctx = N.lib(), self.dev.ctx
        nk, no = ctypes.c_uint64(0), ctypes.c_uint64(0)
        work = (c_void_p(self.work.ptr), self.work_bytes)
        if not self.overlap:
            sh = self.loader.load()
            N.check(ctx, L.kman_groups(ctx, c_void_p(sh.codes.ptr), sh.n_own, self.k, self.flags, self.m, *work,
                                       c_void_p(self.out_keys.ptr), c_void_p(self.out_vals.ptr), self.vb, byref(nk),
                                       byref(no)), "kman_groups")
        else:
            n_all = self.n_bases
            codes = c_void_p(self.loader.shard.codes.ptr)
            nt, tb = ctypes.c_uint32(0), ctypes.c_uint64(0)
            N.check(ctx, L.kman_groups_begin(ctx, n_all, self.k, self.flags, self.m, *work, byref(nt), byref(tb)),
                    "kman_groups_begin")
            width = int(tb.value)

            def on_chunk(n: int) -> None:
                if width and n >= 64 + width:  # tile t reads codes below (t + 1) * width + 64
                    N.check(ctx, L.kman_groups_extract(ctx, codes, n_all, self.k, self.flags, self.m, *work,
                                                       (n - 64) // width), "kman_groups_extract")

            sh = self.loader.load(on_chunk)
            if sh.n_own != n_all:
                raise RuntimeError("the input changed size (%d -> %d bases)" % (n_all, sh.n_own))
            N.check(ctx, L.kman_groups_end(ctx, codes, n_all, self.k, self.flags, self.m, *work,
                                           c_void_p(self.out_keys.ptr), c_void_p(self.out_vals.ptr), self.vb,
                                           byref(nk), byref(no)), "kman_groups_end")
        self.n_kmers, self.n_out = int(nk.value), int(no.value)
        return self.n_kmers

    def free(self) -> None:
        for b in (self.work, self.out_keys, self.out_vals):
            b.free()
        self.loader.free()
