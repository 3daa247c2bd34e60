"""Record types of the k-mer path: coordinates, k-mers, sequence counts.

Mirrors the names and behaviour of kmermaid/seq.py (reference) so callers of
the reference find the same surface:

* ``SequenceCoords`` — ``ref:start-end:strand`` headers (seq.py:15-127),
  same validation (AssertionError on negative coordinates / bad strand) and
  the same parse regex (seq.py:44-48).
* ``KMer`` — header + sequence record (seq.py:415-509).
* ``SequenceCount`` — sequence + list of headers (seq.py:512-565).
* ``Sequence`` — nucleic-acid sequence with k-mer generators
  (seq.py:130-412).  ``kmerator`` / ``yield_kmers`` run the window
  enumeration on the GPU (kman_extract) and only build the Python objects on
  the host.

The alphabet of ``oligo_melting`` (un-vendored reference dependency,
github.com/ggirelli/oligo-melting rev 301b2c8) is restated as the reference's
own tests pin it: DNA "ACGT" / complement "TGCA" (tests/test_seq.py:152-181).
"""

from __future__ import annotations

import logging
import re
from enum import Enum, unique
from typing import Iterator, List, Tuple


@unique
class NATYPES(Enum):
    """Nucleic-acid types (oligo_melting.NATYPES)."""

    DNA = 1
    RNA = 2


AB_NA = {NATYPES.DNA: ["ACGT", "TGCA"], NATYPES.RNA: ["ACGU", "UGCA"]}


class SequenceCoords:
    """Reference window coordinates ``ref:start-end:strand`` (0-based, half-open,
    always on the + strand; seq.py:15-127)."""

    @unique
    class STRAND(Enum):
        PLUS = 0
        MINUS = 1

        @property
        def label(self) -> str:
            return "+-"[int(self.value)]

    regexp = re.compile(r"^(?P<ref>.+):(?P<start>[0-9]+)-(?P<end>[0-9]+):(?P<strand>[\+-])$")

    def __init__(self, ref: str, start: int, end: int, strand: "SequenceCoords.STRAND" = STRAND.PLUS):
        if start < 0:
            raise AssertionError
        if end < 0:
            raise AssertionError
        if not isinstance(strand, self.STRAND):
            raise AssertionError
        self._ref, self._start, self._end, self._strand = ref, start, end, strand

    ref = property(lambda self: self._ref)
    start = property(lambda self: self._start)
    end = property(lambda self: self._end)
    strand = property(lambda self: self._strand)

    def __eq__(self, other):
        return (
            isinstance(other, SequenceCoords)
            and self.ref == other.ref
            and self.start == other.start
            and self.end == other.end
            and self.strand == other.strand
        )

    @staticmethod
    def rev(strand: "SequenceCoords.STRAND") -> "SequenceCoords.STRAND":
        if strand == SequenceCoords.STRAND.PLUS:
            return SequenceCoords.STRAND.MINUS
        return SequenceCoords.STRAND.PLUS

    def __repr__(self):
        return "%s:%d-%d:%s" % (self.ref, self.start, self.end, self.strand.label)

    @staticmethod
    def from_str(s: str) -> "SequenceCoords":
        m = SequenceCoords.regexp.search(s)
        if m is None:
            raise AssertionError(f"incompatible string: {s}")
        strand = SequenceCoords.STRAND.PLUS if m.group("strand") == "+" else SequenceCoords.STRAND.MINUS
        return SequenceCoords(m.group("ref"), int(m.group("start")), int(m.group("end")), strand)


def _check_ab(s: str, ab: List[str]) -> bool:
    return all(c in ab[0] for c in s)


def _mkrc(s: str, t: NATYPES) -> str:
    ab = AB_NA[t]
    return s[::-1].translate(str.maketrans(ab[0], ab[1]))


class Sequence:
    """Nucleic-acid sequence (oligo_melting.Sequence + seq.py:130-412)."""

    doReverseComplement = False

    def __init__(self, seq: str, t: NATYPES, name=None):
        if not isinstance(t, NATYPES):
            raise AssertionError("sequence type must be from NATYPES")
        self.text = seq.upper()
        self.natype = t
        self.name = name
        self.ab = AB_NA[t]

    def __eq__(self, other):
        return self.text == other.text and self.natype == other.natype

    check_ab = staticmethod(_check_ab)
    mkrc = staticmethod(_mkrc)

    def kmers(self, k: int) -> Iterator["KMer"]:
        return self.kmerator(self.text, k, self.natype, self.name, rc=self.doReverseComplement)

    def batches(self, k: int, batchSize: int) -> Iterator[Tuple[str, int]]:
        return self.batcher(self.text, k, batchSize)

    def kmers_batched(self, k: int, batchSize: int = 1) -> Iterator[Iterator["KMer"]]:
        if batchSize < 1:
            raise AssertionError
        if batchSize == 1:
            yield self.kmers(k)
        else:
            yield from self.kmerator_batched(self.text, k, self.natype, batchSize, self.name,
                                             rc=self.doReverseComplement)

    @staticmethod
    def yield_kmers(seq: str, prefix: str, k: int, t: NATYPES, offset: int,
                    strand: SequenceCoords.STRAND, rc: bool) -> Iterator["KMer"]:
        """Every valid window of ``seq`` as KMer(s), in the reference's order
        (seq.py:285-328).  The windows and their 2-bit keys come from the GPU
        extract kernel; skipped windows are logged like the reference."""
        if t != NATYPES.DNA:
            raise NotImplementedError("the MI355X path enumerates DNA k-mers (the reference CLI is DNA-only)")
        from . import engine

        up = seq.upper()
        keys, pos = engine.kmers_of_sequence(up, k, rc)
        if len(up) >= k and len(keys) < (len(up) - k + 1) * (2 if rc else 1):
            valid = set(int(p) >> 1 for p in pos)
            for i in range(len(up) - k + 1):
                if i not in valid:
                    logging.warning("skipped sequence with unexpected character: " + up[i : i + k])
        minus = SequenceCoords.STRAND.MINUS if strand == SequenceCoords.STRAND.PLUS else SequenceCoords.STRAND.PLUS
        for key, p in zip(keys.tolist(), pos.tolist()):
            i = p >> 1
            s = strand if not (p & 1) else minus
            yield KMer(prefix, i + offset, i + offset + k, engine.decode_key(key, k), t, strand=s)

    @staticmethod
    def kmerator(seq: str, k: int, t: NATYPES, prefix: str = "ref", offset: int = 0,
                 strand: SequenceCoords.STRAND = SequenceCoords.STRAND.PLUS, rc: bool = False) -> Iterator["KMer"]:
        return iter(Sequence.yield_kmers(seq, prefix, k, t, offset, strand, rc))

    @staticmethod
    def batcher(seq: str, k: int, batchSize: int) -> Iterator[Tuple[str, int]]:
        """Overlapping chunks for k-mer batching (seq.py:362-383).  The
        reference loops forever when batchSize < k (§A-6); here that is an
        AssertionError."""
        if batchSize < k:
            raise AssertionError("batchSize must be >= k")
        start = 0
        while start < len(seq) - k + 1:
            end = min(len(seq), start + batchSize)
            yield (seq[start:end], start)
            start += batchSize - k + 1

    @staticmethod
    def kmerator_batched(seq: str, k: int, t: NATYPES, batchSize: int = 1, prefix="ref",
                         rc=False) -> Iterator[Iterator["KMer"]]:
        if batchSize < 1:
            raise AssertionError
        if batchSize == 1:
            yield Sequence.kmerator(seq, k, t, prefix, rc=rc)
            return  # the reference falls through here (§A-6); this is the evident intent
        for chunk, i in Sequence.batcher(seq, k, batchSize):
            yield Sequence.kmerator(chunk, k, t, prefix, offset=i, rc=rc)


class KMer(Sequence):
    """A k-mer with its coordinates (seq.py:415-509)."""

    def __init__(self, chrom: str, start: int, end: int, seq: str, t: NATYPES = NATYPES.DNA,
                 strand: SequenceCoords.STRAND = SequenceCoords.STRAND.PLUS):
        if len(seq) != end - start:
            raise AssertionError
        super().__init__(seq, t)
        self._coords = SequenceCoords(chrom, start, end, strand)

    coords = property(lambda self: self._coords)
    header = property(lambda self: str(self._coords))
    seq = property(lambda self: self.text)

    def __eq__(self, other):
        return self.coords == other.coords and super().__eq__(other)

    @staticmethod
    def from_fasta(record: Tuple[str, str], t: NATYPES = NATYPES.DNA) -> "KMer":
        c = SequenceCoords.from_str(record[0])
        return KMer(c.ref, c.start, c.end, record[1], t, strand=c.strand)

    from_file = from_fasta

    def as_fasta(self) -> str:
        return ">%s\n%s\n" % (self.header, self.seq)

    def __repr__(self):
        return "%s\t%s" % (self.header, self.seq)

    def is_ab_checked(self) -> bool:
        return all(c in self.ab[0] for c in set(self.text))


class SequenceCount(Sequence):
    """A sequence and the headers of the records carrying it (seq.py:512-565)."""

    def __init__(self, seq, headers, t=NATYPES.DNA):
        super().__init__(seq, t)
        if not all(isinstance(h, str) for h in headers):
            raise AssertionError
        self.__headers = list(headers)

    header = property(lambda self: self.__headers.copy())
    seq = property(lambda self: self.text)

    @staticmethod
    def from_text(line: str, t: NATYPES = NATYPES.DNA) -> "SequenceCount":
        seq, headers = line.strip().split("\t")
        return SequenceCount(seq, headers.split(" "), t)

    from_file = from_text

    def __repr__(self) -> str:
        return "%s\t%s" % (self.seq, " ".join(self.header))

    def as_text(self) -> str:
        return str(self) + "\n"
