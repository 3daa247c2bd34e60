"""Chunk 3 of the streamed loader parses wrong (debug): codes prefilled,
then the chunk parsed alone."""
import sys
from ctypes import byref, c_void_p

import numpy as np

sys.path.insert(0, "tests/golden")
sys.path.insert(0, ".")
import inputs  # noqa: E402

from kman_amd import _native as N  # noqa: E402
from kman_amd import engine, shard  # noqa: E402

dev = engine.default_device()
text = inputs.syn_numpy(3_000_000, 11, record_len=700_000, width=61)
p = engine.parse(dev, text)
want = dev.download(p.codes, p.n_bases, np.uint8)
lo, hi = 1000098, 1333472
chunk = text[lo:hi]
exp = np.frombuffer(chunk.replace(b"\n", b""), np.uint8)
print("expected bases", len(exp), "at", 983955, flush=True)
for fill in (0xEE, 0x00, 0xEE):
    t = dev.alloc(len(chunk) + 64 + 4096)
    dev.memset(t, 0x41 if fill else 0x0A, len(chunk) + 64 + 4096)
    dev.upload(t, chunk)
    OFF = 983955
    c = dev.alloc(OFF + len(exp) + 4096)
    dev.memset(c, fill, OFF + len(exp) + 4096)
    hd, sq = dev.alloc(8 * 1024), dev.alloc(8 * 1024)
    info = N.ParseInfo()
    N.check(dev.ctx, N.lib().kman_parse_fasta_at(dev.ctx, c_void_p(t.ptr), len(chunk), N.KMAN_PARSE_IN_RECORD,
                                                 c_void_p(c.ptr), OFF, c_void_p(hd.ptr), c_void_p(sq.ptr), 1024,
                                                 byref(info)), "parse")
    got = dev.download(c, int(info.n_bases), np.uint8, offset=OFF)
    w = want[983955:983955 + len(got)]
    bad = np.nonzero(got != w)[0]
    print("fill", hex(fill), "n_bases", info.n_bases, "bad", len(bad), bad[:3], bad[-3:], flush=True)
    if len(bad):
        print(" got", got[bad[:8]], "want", w[bad[:8]], flush=True)
    for b in (t, c, hd, sq):
        b.free()
