"""Batch: a fixed-capacity group of records (kmermaid/batch.py:19-395).

Two storage modes share the reference's surface (``size``, ``current_size``,
``remaining``, ``tmp``, ``is_written``, ``add``, ``record_gen``, ``sorted``,
``write``, ``unwrite``, ``reset``, ``from_file``, ...):

* device mode — a view ``[start, end)`` of a device-resident k-mer stream
  (``source.FastaSource``) created by ``FastaBatcher.do``.  Sorting runs on the
  GPU (``kman_sort``), the batch FASTA is formatted by ``kman_format_uniq``;
  nothing is spilled to disk unless ``write()`` / ``copy_batches`` asks for it.
* host mode — the reference's generic in-memory container for arbitrary
  record types (its own tests use ``str`` records), spilled to a temp file on
  ``write()``.  This is container bookkeeping, not k-mer arithmetic.
"""

from __future__ import annotations

import gzip
import os
import random
import tempfile
import time
from typing import IO, Any, Iterator, List, Optional, Type

from .seq import KMer


class Batch:
    _fread = "from_file"
    _fwrite = "as_fasta"
    _keyAttr = "seq"
    isFasta = True
    suffix = ".fa"

    def __init__(self, t: Type, tmpDir: str, size: int = 1, _records: bool = True):
        if size < 1:
            raise AssertionError
        self.__size = int(size)
        self._remaining = self.__size
        self.__type = t
        self._tmp_dir = tmpDir
        self._tmp: Optional[str] = None
        self._written = False
        self._i = 0
        # (a device batch holds no record list: from_source skips the
        # size-long list, 0.26 s for config 2's 1000 batches of 1 M)
        self.__records: Optional[List[Any]] = [None] * self.__size if _records else None
        # device mode
        self._src = None
        self._start = 0
        self._end = 0
        self._sorted_view = False

    # --------------------------------------------------------- device mode
    @classmethod
    def from_source(cls, src, start: int, end: int, size: int, tmpDir: str) -> "Batch":
        b = cls(KMer, tmpDir, size, _records=False)
        b._src, b._start, b._end = src, int(start), int(end)
        b._i = int(end - start)
        b._remaining = b.size - b._i
        b.__records = None
        return b

    @property
    def on_device(self) -> bool:
        return self._src is not None

    @property
    def source(self):
        return self._src

    @property
    def stream_range(self):
        return self._start, self._end

    # ------------------------------------------------------------ properties
    @property
    def is_written(self) -> bool:
        return self._written

    @property
    def current_size(self) -> int:
        return self._i

    @property
    def size(self) -> int:
        return self.__size

    @property
    def remaining(self) -> int:
        return self._remaining

    @property
    def collection(self):
        if self.__records is None:
            return None
        return self.__records.copy()

    @property
    def type(self):
        return self.__type

    @property
    def tmp(self) -> str:
        """Temp file name (batch.py:96-106: prefix hash(time), random, suffix)."""
        if self._tmp is None:
            d = self._tmp_dir or tempfile.gettempdir()
            while True:
                name = os.path.join(d, "%d%08x%s" % (hash(time.time()), random.getrandbits(32), self.suffix))
                if not os.path.exists(name):
                    break
            self._tmp = name
        return self._tmp

    @property
    def info(self) -> str:
        info = "%s\ntype: %s\nsize: %d" % (self.tmp, self.type, self.size)
        info += "\ni: %d\nremaining: %d" % (self.current_size, self.remaining)
        info += "\nwritten: %r\n" % self.is_written
        return info

    def _check_attr(self, name):
        if not isinstance(name, str) or not hasattr(self.type, name):
            raise AssertionError
        return name

    keyAttr = property(lambda self: self._keyAttr, lambda self, k: setattr(self, "_keyAttr", self._check_attr(k)))
    fread = property(lambda self: self._fread, lambda self, f: setattr(self, "_fread", self._check_attr(f)))
    fwrite = property(lambda self: self._fwrite, lambda self, f: setattr(self, "_fwrite", self._check_attr(f)))

    # ---------------------------------------------------------- records
    def _device_sorted(self, want_pos: bool = True):
        from .source import download_sorted

        return download_sorted(self._src, self._start, self._end, want_pos)

    def sorted(self, smart: bool = False) -> Any:
        """Records sorted by sequence, ties in stream order (batch.py:156-168)."""
        if self.on_device:
            return list(self._kmers_from(*self._device_sorted()))
        if self.isFasta:
            return sorted(self.record_gen(smart), key=lambda x: getattr(x, self.keyAttr))
        return sorted(self.record_gen(smart))

    def _kmers_from(self, keys, pos) -> Iterator[KMer]:
        from .engine import decode_key, decode_words
        from .seq import SequenceCoords

        k = self._src.k
        dec = (lambda x: decode_words(x, k)) if keys.ndim == 2 else (lambda x: decode_key(x, k))
        for key, p in zip(keys.tolist(), pos.tolist()):
            c = SequenceCoords.from_str(self._src.header(p))
            yield KMer(c.ref, c.start, c.end, dec(key), strand=c.strand)

    def _record_gen_from_handle(self, TH: IO, smart: bool = False) -> Iterator[Any]:
        if self.isFasta:
            title, seq = None, []
            for line in TH:
                if line.startswith(">"):
                    if title is not None:
                        yield getattr(self.type, self.fread)((title, "".join(seq)))
                    title, seq = line[1:].rstrip(), []
                elif title is not None:
                    seq.append(line.rstrip())
            if title is not None:
                yield getattr(self.type, self.fread)((title, "".join(seq)))
        else:
            for line in TH:
                yield getattr(self.type, self.fread)(line)

    def _record_gen_from_file(self, smart: bool = False) -> Iterator[Any]:
        TH = gzip.open(self.tmp, "rt") if self.tmp.endswith(".gz") else open(self.tmp, "r")
        with TH:
            yield from self._record_gen_from_handle(TH, smart)

    def record_gen(self, smart: bool = False) -> Iterator[Any]:
        if self.is_written:
            yield from self._record_gen_from_file(smart)
        elif self.on_device:
            # after FastaBatcher.do every batch is stored sorted (batcher.py:392)
            yield from self._kmers_from(*self._device_sorted())
        else:
            for record in self.__records:
                if record is not None:
                    yield record

    def check_record(self, record: Any) -> None:
        if type(record) != self.type:
            raise AssertionError(f"record must be {self.type}, not {type(record)}.")

    def add(self, record: Any) -> None:
        if self.is_full():
            raise AssertionError("this batch is full.")
        if self.is_written:
            raise AssertionError("this batch has been stored locally.")
        if self.on_device:
            raise AssertionError("device batches are filled by FastaBatcher.do")
        self.check_record(record)
        self.__records[self._i] = record
        self._i += 1
        self._remaining -= 1

    def add_all(self, recordGen) -> None:
        for record in recordGen:
            self.add(record)

    def to_write(self, doSort: bool = False) -> List[Any]:
        gen = self.sorted() if doSort else self.record_gen()
        return [getattr(r, self.fwrite)() for r in gen if r is not None]

    def fasta_bytes(self) -> bytes:
        """The batch's sorted FASTA bytes, formatted from device results."""
        keys, pos = self._device_sorted()
        return self._src.format_fasta(keys, pos)

    def write(self, doSort: bool = False, force: bool = False) -> None:
        if self.is_written and not force:
            return
        if self.on_device:
            data = self.fasta_bytes()
            with open(self.tmp, "wb") as fh:
                fh.write(data)
        else:
            output = [x if x.endswith("\n") else x + "\n" for x in self.to_write(doSort)]
            with open(self.tmp, "w") as TH:
                TH.write("".join(output))
            self.__records = [None]
        self._written = True

    @staticmethod
    def from_file(path: str, t: Type = KMer, isFasta: bool = True, smart: bool = False,
                  reSort: bool = False) -> "Batch":
        """Link an existing batch file (batch.py:298-344)."""
        opener = gzip.open if path.endswith(".gz") else open
        with opener(path, "rt") as FH:
            if isFasta:
                size = max(2, sum(1 for line in FH if line.startswith(">")))
            else:
                size = max(2, sum(1 for _ in FH))
        batch = Batch(t, os.path.dirname(path), size)
        batch._tmp = path
        batch._i = size
        batch._remaining = 0
        batch._written = True
        batch.isFasta = isFasta
        if reSort:
            batch.write(doSort=True, force=True)
        return batch

    @staticmethod
    def from_batcher(batch_type: Type, size: int = 1, tmp: Optional[str] = None) -> "Batch":
        if size < 1:
            raise AssertionError(f"size cannot be 0 or negative: {size}")
        return Batch(batch_type, tmp or tempfile.gettempdir(), size)

    def reset(self) -> None:
        if self.is_written and os.path.isfile(self.tmp):
            os.remove(self.tmp)
        self._written = False
        self._src = None
        self._i = 0
        self._remaining = self.size
        self.__records = [None] * self.size

    def is_full(self) -> bool:
        return self.remaining == 0

    def unwrite(self) -> None:
        if not self.is_full() and self.is_written and not self.on_device:
            recs = list(self.record_gen())
            self.__records = [None] * self.size
            self.__records[: self.current_size] = recs
            self._written = False
            os.remove(self.tmp)
