"""One process per GPU behind the drop-in surface.

Launched N times with ``WORLD_SIZE`` / ``RANK`` / ``LOCAL_RANK`` in the
environment (``python -m torch.distributed.run --nproc-per-node N -m
kman_amd count IN OUT 21``, or any launcher that sets them before the first
GPU call), the ``kmer`` CLI and the reference's operator surface
(``FastaBatcher(...).do(IN, k).collection`` -> ``KJoinerThreading.join``,
kmermaid/scripts/kmer_count.py:100-120, kmer_uniq.py:73-92) run the
multi-GPU join of SURVEY §8e instead of N copies of the single-GPU one:

* ``FastaBatcher.do`` on rank q loads only its byte range of the FASTA (cut at
  line starts, plus a (k-1)-base halo: kman_amd/shard.py) onto GPU
  ``LOCAL_RANK`` and hands back ONE batch, the rank's windows
  (``ShardedSource``);
* ``KJoiner.join`` on that batch builds the RCCL communicator (rank 0 writes
  the 128-byte id to a file next to the output), runs the key rounds of
  ``dist.DistPipeline`` (shard histogram, all-gathered bucket totals, per
  round one RCCL all-to-all of packed items, per-bucket passes + LDS finish)
  and writes the reference's bytes into ONE output file, every rank its
  slice at its offset (``DistPipeline.emit_gen``);
* ``kmer hist`` runs canonical counting + the all-reduced spectrum.

Outside the multi-GPU domain (k > 32, ``-B`` reloads, VEC_* modes, ``kmer
batch``) rank 0 runs the single-GPU path on the whole input and the other
ranks leave without output: the result is the same file.  ``KMAN_DIST=1``
forces the multi-GPU path at world size 1 (RCCL with one rank: tests);
``KMAN_DIST=0`` turns it off.
"""

from __future__ import annotations

import gzip
import logging
import mmap
import os
import secrets
import struct
import tempfile
import time
from typing import Callable, Optional, Tuple

import numpy as np

from . import engine

_MAGIC = b"KMANRCID"
_START = time.time()


def world_env() -> Tuple[int, int, int]:
    """(world size, rank, local rank) from the launcher's environment."""
    w = int(os.environ.get("WORLD_SIZE", "1") or 1)
    r = int(os.environ.get("RANK", "0") or 0)
    loc = int(os.environ.get("LOCAL_RANK", str(r)) or 0)
    if w < 1 or not 0 <= r < w:
        raise RuntimeError("bad launcher environment: WORLD_SIZE=%d RANK=%d" % (w, r))
    return w, r, loc


def distributed() -> bool:
    """True when this process is one rank of a multi-GPU run (or KMAN_DIST=1)."""
    env = os.environ.get("KMAN_DIST")
    if env is not None:
        return env == "1"
    return world_env()[0] > 1


def solo_rank() -> bool:
    """For work outside the multi-GPU domain: True on the rank that does it
    alone (rank 0), False on the others (they leave without output)."""
    w, r, _ = world_env()
    return w == 1 or r == 0


class FileReader:
    """A shard.py reader over a FASTA file: plain files memory-mapped (a rank
    touches only its byte range and the cuts around it).  Gzip input
    (batcher.py:480 opens ``.gz`` with gzip.open): one rank decompresses it
    in memory; under a multi-GPU launch rank 0 decompresses it ONCE, as a
    stream, into a temp file that every rank then memory-maps like a plain
    one (so no rank holds the whole text, and the file is inflated once, not
    once per rank).  Rank 0 removes the temp file when it closes the reader
    (the peers' maps stay valid) or at exit."""

    def __init__(self, path: str, world: int = 1, rank: int = 0, directory: Optional[str] = None,
                 timeout: Optional[float] = None):
        self._fh = self._mm = None
        self._tmp = None
        # where rank 0 inflates a gzip input, and how long the peers wait for
        # it (rank 0 marks a failure at once, so the wait only bounds a rank 0
        # that died without a word)
        directory = directory or os.environ.get("KMAN_GZ_DIR") or None
        if timeout is None:
            timeout = float(os.environ.get("KMAN_GZ_TIMEOUT", "1800"))
        if path.endswith(".gz") and world > 1:
            path = self._gunzip_shared(path, world, rank, directory, timeout)
        if path.endswith(".gz"):
            with gzip.open(path, "rb") as fh:
                self._mv = memoryview(fh.read())
        else:
            self._fh = open(path, "rb")
            size = os.fstat(self._fh.fileno()).st_size
            if size:
                self._mm = mmap.mmap(self._fh.fileno(), 0, access=mmap.ACCESS_READ)
                self._mv = memoryview(self._mm)
            else:
                self._mv = memoryview(b"")
        self.size = len(self._mv)

    def _gunzip_shared(self, path: str, world: int, rank: int, directory: Optional[str], timeout: float,
                       skew: float = 30.0) -> str:
        """The plain text of `path` in a temp file shared by the ranks of this
        launch (keyed like the RCCL id file, plus the input's identity); rank 0
        writes it and then a marker holding its start time, a peer accepts
        only a marker written by a rank 0 that started no earlier than `skew`
        seconds before itself."""
        import atexit
        import shutil
        import zlib

        st = os.stat(path)
        ident = "%08x" % (zlib.crc32(("%s|%d|%d" % (os.path.abspath(path), st.st_size, st.st_mtime_ns)).encode())
                          & 0xffffffff)
        plain = _id_path("gz" + ident, directory) + ".fa"
        done = plain + ".done"
        def mark(status: bytes) -> None:  # MAGIC | rank 0's start | status (b"ok" or b"!" + error text)
            with open(done + ".tmp", "wb") as fh:
                fh.write(_MAGIC + struct.pack("<d", _START) + status)
            os.replace(done + ".tmp", done)

        if rank == 0:
            for q in (done, plain):
                try:
                    os.remove(q)
                except OSError:
                    pass
            part = plain + ".part%d" % os.getpid()
            self._tmp = (plain, done)
            atexit.register(self._remove_tmp)
            try:
                # the inflated size (gzip's ISIZE trailer: the size mod 2^32, so
                # at least that much) must fit the directory's free space
                with open(path, "rb") as fh:
                    fh.seek(-4, os.SEEK_END)
                    (isize,) = struct.unpack("<I", fh.read(4))
                free = shutil.disk_usage(os.path.dirname(plain)).free
                if isize > free:
                    raise OSError("inflating %s needs >= %d bytes in %s, %d free (set KMAN_GZ_DIR)"
                                  % (path, isize, os.path.dirname(plain), free))
                with gzip.open(path, "rb") as src, open(part, "wb") as dst:
                    shutil.copyfileobj(src, dst, 16 << 20)
                os.replace(part, plain)
            except BaseException as e:
                # the peers read the failure at once instead of waiting out
                # their timeout
                try:
                    mark(b"!" + ("%s: %s" % (type(e).__name__, e)).encode("utf-8", "replace")[:4000])
                    self._tmp = (plain,)  # (the marker outlives this process: a peer may start polling later)
                except OSError:
                    pass
                raise
            finally:
                try:
                    os.remove(part)
                except OSError:
                    pass
            mark(b"ok")
            return plain
        t0 = time.time()
        while True:
            try:
                with open(done, "rb") as fh:
                    blob = fh.read()
                if blob[:8] == _MAGIC and len(blob) >= 16 and struct.unpack("<d", blob[8:16])[0] >= _START - skew:
                    if blob[16:17] == b"!":
                        raise RuntimeError("rank %d: rank 0 failed to decompress %s: %s"
                                           % (rank, path, blob[17:].decode("utf-8", "replace")))
                    return plain
            except OSError:
                pass
            if time.time() - t0 > timeout:
                raise RuntimeError("rank %d: rank 0 did not decompress %s into %s within %.0f s (KMAN_GZ_TIMEOUT)"
                                   % (rank, path, plain, timeout))
            time.sleep(0.05)

    def _remove_tmp(self) -> None:
        if self._tmp:
            for q in self._tmp:
                try:
                    os.remove(q)
                except OSError:
                    pass
            self._tmp = None

    def read(self, lo: int, hi: int) -> bytes:
        return bytes(self._mv[max(0, lo):max(0, min(hi, self.size))])

    def close(self) -> None:
        self._mv.release()
        if self._mm is not None:
            self._mm.close()
            self._mm = None
        if self._fh is not None:
            self._fh.close()
            self._fh = None
        self._remove_tmp()


def launch_nonce() -> str:
    """Something every rank of ONE launch shares (and, where the launcher
    offers it, the next launch does not), taken from the environment only:
    the launcher's run id (KMAN_RUN_ID, set by bench.py's spawner), else
    torch.distributed.run's TORCHELASTIC_RUN_ID with its restart count when
    the id is not the constant "none", else empty -- the start-time check in
    `rendezvous` then tells launches apart.  (Not the parent PID: a worker
    wrapped in a shell or launcher has a parent of its own, and its peers
    would wait on another file.)"""
    rid = os.environ.get("KMAN_RUN_ID")
    if rid:
        return rid
    tid = os.environ.get("TORCHELASTIC_RUN_ID", "")
    if tid and tid != "none":
        return "%s-%s" % (tid, os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
    # torch.distributed.run with the default run id "none": its per-launch log
    # directory (<tmp>/torchelastic_<random>/<run id>_<random>/attempt_<n>/<local
    # rank>/error.json) is shared by the workers of one launch and by no other
    ef = os.environ.get("TORCHELASTIC_ERROR_FILE", "")
    if ef and ef != os.devnull:
        import zlib

        attempt = os.path.dirname(os.path.dirname(ef))
        return "te%08x" % (zlib.crc32(attempt.encode()) & 0xffffffff)
    return ""


def _id_path(tag: str, directory: Optional[str] = None) -> str:
    key = "%s_%s_%s_%s" % (os.environ.get("MASTER_PORT", "0"), launch_nonce(), os.environ.get("WORLD_SIZE", "1"),
                           tag)
    return os.path.join(directory or tempfile.gettempdir(), "kman_rccl_id_" + key.replace(os.sep, "_"))


def rendezvous(rank: int, world: int, tag: str = "0", make_uid: Optional[Callable[[], bytes]] = None,
               directory: Optional[str] = None, timeout: float = 300.0, skew: float = 30.0) -> bytes:
    """The 128-byte RCCL id, shared through a file (one node: every rank
    sees the same temp dir).  Rank 0 removes any file a crashed launch left
    on the same key, then writes MAGIC | its start time | a nonce | the id
    atomically; a peer accepts only a file whose writer started no earlier
    than `skew` seconds before the peer itself (the ranks of one launch start
    together), so a stale id is never used."""
    if make_uid is None:
        from . import dist

        make_uid = dist.unique_id
    if world == 1:
        return make_uid()
    path = _id_path(tag, directory)
    if rank == 0:
        try:
            os.remove(path)
        except OSError:
            pass
        uid = make_uid()
        blob = _MAGIC + struct.pack("<d", _START) + secrets.token_bytes(8) + uid
        with open(path + ".tmp%d" % os.getpid(), "wb") as fh:
            fh.write(blob)
        os.replace(path + ".tmp%d" % os.getpid(), path)
        return uid
    t0 = time.time()
    while True:
        try:
            with open(path, "rb") as fh:
                blob = fh.read()
            if blob[:8] == _MAGIC and len(blob) >= 24 + 128:
                (started,) = struct.unpack("<d", blob[8:16])
                if started >= _START - skew:
                    return blob[24:24 + 128]
        except OSError:
            pass
        if time.time() - t0 > timeout:
            raise RuntimeError("rank %d: no RCCL id from rank 0 at %s" % (rank, path))
        time.sleep(0.05)


def remove_id(tag: str = "0", directory: Optional[str] = None) -> None:
    try:
        os.remove(_id_path(tag, directory))
    except OSError:
        pass


class ShardedSource:
    """This rank's byte range of ONE FASTA on GPU LOCAL_RANK (the k-mer
    stream of FastaBatcher.do under a multi-process launch): codes of the
    rank's bytes + a (k-1)-base halo, its record table, its window count.
    ``join`` runs the multi-GPU count / uniq into one output file."""

    _joins = 0

    def __init__(self, dev: engine.Device, path: str, k: int, rc: bool):
        from ctypes import byref, c_uint64, c_void_p

        from . import _native as N
        from . import shard as S

        engine._check_k(k)
        self.world, self.rank, self.local = world_env()
        self.dev, self.k, self.rc, self.path = dev, k, rc, path
        self.reader = FileReader(path, self.world, self.rank)
        self.spec = S.shard_specs(self.reader, self.world, k)[self.rank]
        self.loader = S.ShardLoader(dev, self.reader, self.spec, k)
        self.shard = self.loader.load()
        out = c_uint64(0)
        if self.shard.n_eff:
            N.check(dev.ctx, N.lib().kman_count_kmers(dev.ctx, c_void_p(self.shard.codes.ptr), self.shard.n_eff, k,
                                                      engine.flags_for(rc, False), byref(out)), "kman_count_kmers")
        self.n_kmers = int(out.value)  # this rank's windows (x2 with -r)

    def _pipe(self, mode: str, canonical: bool = False, ordered: bool = True):
        from . import dist

        ShardedSource._joins += 1
        tag = "join%d" % ShardedSource._joins
        uid = rendezvous(self.rank, self.world, tag)
        pipe = dist.DistPipeline(self.dev, None, self.k, mode, self.world, self.rank, uid, canonical=canonical,
                                 rc=self.rc and not canonical, shard=self.shard, ordered=ordered)
        if self.rank == 0:
            remove_id(tag)  # (every rank has joined the communicator)
        return pipe

    def join(self, count: bool, outpath: str) -> int:
        """Count / uniq of the whole FASTA across the ranks into `outpath`
        (every rank writes its slice); returns the file's size."""
        pipe = self._pipe("count" if count else "uniq")
        try:
            pipe.step()
            return pipe.comm.run(pipe.emit_gen(outpath))
        finally:
            pipe.free()

    def hist(self, nbins: int, canonical: bool = True) -> np.ndarray:
        """Abundance spectrum of the whole FASTA (canonical keys by default),
        all-reduced: every rank gets it."""
        pipe = self._pipe("count", canonical=canonical, ordered=False)
        try:
            pipe.step()
            return pipe.comm.run(pipe.hist_gen(nbins))
        finally:
            pipe.free()

    # the per-batch surface needs the global stream, which no rank holds
    def kmers(self, want_pos: bool):
        raise NotImplementedError("a rank's shard batch under a multi-GPU launch only joins (KJoiner.join); "
                                  "per-batch sort / record_gen need the single-GPU path (WORLD_SIZE=1)")

    def header(self, pos: int) -> str:
        return self.kmers(False)

    def format_fasta(self, keys, pos) -> bytes:
        return self.kmers(False)

    def free(self) -> None:
        if self.loader is not None:
            self.loader.free()
            self.loader = None
        self.reader.close()


def log_solo(what: str) -> None:
    w, r, _ = world_env()
    if w > 1 and r != 0:
        logging.info("rank %d of %d: %s runs on rank 0 alone" % (r, w, what))
