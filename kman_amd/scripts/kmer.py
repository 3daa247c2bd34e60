"""``kmer`` command group: batch / count / uniq (kmermaid/scripts/*.py).

Same arguments, flags, defaults, outputs and errors as the reference CLI; the
work runs on the GPU through kman_amd (FastaBatcher.do + KJoiner.join).
"""

from __future__ import annotations

import logging
import os
import resource
import tempfile
import warnings
from typing import Optional

import click

from .. import __version__, engine, launch
from ..batcher import BatcherThreading, FastaBatcher, load_batches
from ..io import copy_batches, input_file_exists, set_tempdir
from ..join import KJoiner, KJoinerThreading
from . import arguments as args

CONTEXT_SETTINGS = dict(help_option_names=["-h", "--help"])

# `kmer count` declares -m twice (batch mode and count mode), exactly like the
# reference (arguments.py:104-115 and 134-149); the later one wins in both.
warnings.filterwarnings("ignore", message="The parameter -m is used more than once")


@click.group(name="kmer", context_settings=CONTEXT_SETTINGS,
             help="K-mer management tools, MI355X engine (kman_amd %s)." % __version__)
@click.version_option(__version__)
def main():
    """Entry point."""


def _batches(input_path, k, reverse, scan_mode, batch_size, batch_mode, threads, tmp, dist=False):
    return (
        FastaBatcher(scan_mode=FastaBatcher.MODE[scan_mode], reverse=reverse, size=batch_size, threads=threads,
                     tmp=tmp, distributed=dist)
        .do(input_path, k, BatcherThreading.FEED_MODE[batch_mode])
        .collection
    )


@main.command(name="count", context_settings=CONTEXT_SETTINGS, help="""
Count occurrences of all k-mers from INPUT.

\b
Counting modes:
       SEQ_COUNT a tabulation-separated table with sequence and count
       VEC_COUNT / VEC_COUNT_MASKED: abundance vectors; like the reference,
                 they raise NotImplementedError, unless KMAN_VEC_COUNT=1
                 selects this engine's vector writer (INTEGRATION.md §4)
The INPUT file can be gzipped.  Launched one process per GPU (WORLD_SIZE >
1), the join runs across the GPUs into one OUTPUT.
""")
@args.input_path()
@args.output_path(file_okay=True)
@args.k()
@args.reverse()
@args.scan_mode()
@args.batch_size()
@args.batch_mode()
@args.previous_batches()
@args.count_mode()
@args.memory_mode()
@args.threads()
@args.tmp()
@args.re_sort()
def count(input_path: str, output_path: str, k: int, reverse: bool = False, scan_mode: str = "KMERS",
          batch_size: int = 1000000, batch_mode: str = "APPEND", previous_batches: Optional[str] = None,
          count_mode: str = "SEQ_COUNT", memory_mode: str = "NORMAL", threads: int = 1,
          tmp: str = tempfile.gettempdir(), re_sort: bool = False) -> None:
    input_file_exists(input_path)
    set_tempdir(tmp)
    dist = _multi_gpu(k, previous_batches, count_mode)
    if dist is None:
        return  # (a rank other than 0, for work outside the multi-GPU domain)
    if previous_batches is not None:
        batches = load_batches(previous_batches, threads, re_sort)
    else:
        batches = _batches(input_path, k, reverse, scan_mode, batch_size, batch_mode, threads, tmp, dist)
    prep_joiner(KJoinerThreading(KJoiner.MODE[count_mode], KJoiner.MEMORY[memory_mode]), len(batches),
                threads).join(batches, output_path)
    logging.info("That's all!")


def _multi_gpu(k: int, previous_batches: Optional[str], count_mode: str = "SEQ_COUNT") -> Optional[bool]:
    """Under a one-process-per-GPU launch (kman_amd/launch.py): True = this
    rank joins across the GPUs; False = the single-GPU path (no launch, or
    rank 0 alone for work outside the multi-GPU domain: k > 32, -B reloads,
    VEC_* modes); None = a rank that leaves that work to rank 0."""
    if not launch.distributed():
        return False
    if k <= 1 or (k <= engine.MAX_K and previous_batches is None and count_mode in ("SEQ_COUNT", "UNIQUE")):
        return True  # (k <= 1 raises in FastaBatcher.do on every rank, as the reference)
    launch.log_solo("k=%d%s%s" % (k, " -B" if previous_batches else "", "" if count_mode == "SEQ_COUNT"
                                  else " " + count_mode))
    return False if launch.solo_rank() else None


def prep_joiner(joiner: KJoinerThreading, n_batches: int, threads: int = 1) -> KJoinerThreading:
    """kmer_count.py:123-144 (the file-descriptor limit is irrelevant on the
    GPU path, but the joiner settings are kept)."""
    joiner.threads = threads
    joiner.batch_size = max(2, int(n_batches / max(1, threads)))
    try:
        lo, hi = resource.getrlimit(resource.RLIMIT_NOFILE)
        joiner.batch_size = min(joiner.batch_size, hi if hi > 0 else joiner.batch_size)
    except (ValueError, OSError):
        pass
    return joiner


@main.command(name="uniq", context_settings=CONTEXT_SETTINGS,
              help="Extract all k-mers that appear only once in the INPUT fasta file.")
@args.input_path()
@args.output_path(file_okay=True)
@args.k()
@args.reverse()
@args.scan_mode()
@args.batch_size()
@args.batch_mode()
@args.previous_batches()
@args.threads()
@args.tmp()
@args.re_sort()
def uniq(input_path: str, output_path: str, k: int, reverse: bool = False, scan_mode: str = "KMERS",
         batch_size: int = 1000000, batch_mode: str = "APPEND", previous_batches: Optional[str] = None,
         threads: int = 1, tmp: str = tempfile.gettempdir(), re_sort: bool = False) -> None:
    input_file_exists(input_path)
    set_tempdir(tmp)
    dist = _multi_gpu(k, previous_batches, "UNIQUE")
    if dist is None:
        return
    if previous_batches is not None:
        batches = load_batches(previous_batches, threads, re_sort)
    else:
        batches = _batches(input_path, k, reverse, scan_mode, batch_size, batch_mode, threads, tmp, dist)
    joiner = KJoinerThreading()
    joiner.threads = threads
    joiner.batch_size = max(2, int(len(batches) / max(1, threads)))
    joiner.join(batches, output_path)
    logging.info("That's all!")


@main.command(name="batch", context_settings=CONTEXT_SETTINGS, help="""
Generate batches of k-mers from an INPUT fasta file.

Batches are written to an OUTPUT folder, which must be empty or non-existent.
The INPUT file can be gzipped.
""")
@args.input_path()
@args.output_path(dir_okay=True)
@args.k()
@args.reverse()
@args.scan_mode()
@args.batch_size()
@args.batch_mode()
@args.threads()
@args.tmp()
@args.compress()
def batch(input_path: str, output_path: str, k: int, reverse: bool = False, scan_mode: str = "KMERS",
          batch_size: int = 1000000, batch_mode: str = "APPEND", threads: int = 1,
          tmp: str = tempfile.gettempdir(), compress: bool = False) -> None:
    input_file_exists(input_path)
    if launch.distributed() and not launch.solo_rank():
        launch.log_solo("kmer batch")  # (the batch files are one stream's consecutive chunks)
        return
    if os.path.isdir(output_path) and len(os.listdir(output_path)) != 0:
        raise AssertionError("output folder must be empty or non-existent.")
    set_tempdir(tmp)
    os.makedirs(output_path, exist_ok=True)
    try:
        copy_batches(_batches(input_path, k, reverse, scan_mode, batch_size, batch_mode, threads, tmp, False),
                     output_path, compress)
    except IOError as e:
        logging.error(f"Unable to write to output directory '{output_path}'.\n{e}")
    logging.info("That's all!")


@main.command(name="hist", context_settings=CONTEXT_SETTINGS, help="""
Abundance spectrum of the (canonical) k-mers of INPUT: one line per
abundance c, "c<TAB>number of distinct k-mers seen c times".

Not part of the reference kman CLI (SURVEY.md §8f-1, BASELINE config 5):
canonical k-mers are min(k-mer, reverse complement); for odd k their counts
are the `kmer count -r` rows whose sequence is <= its reverse complement.
The INPUT file can be gzipped.
""")
@args.input_path()
@args.output_path(file_okay=True)
@args.k()
@click.option("--forward", is_flag=True, help="Count forward k-mers instead of canonical ones.")
@click.option("--max-count", type=click.INT, default=10000, show_default=True,
              help="Abundances from this one up share the last line (>=N).")
def hist(input_path: str, output_path: str, k: int, forward: bool = False, max_count: int = 10000) -> None:
    input_file_exists(input_path)
    if k <= 1:
        raise AssertionError("k must be >= 1, got %d instead." % k)
    if launch.distributed() and k > engine.MAX_K and not launch.solo_rank():
        launch.log_solo("kmer hist k=%d" % k)
        return
    if launch.distributed() and k <= engine.MAX_K:
        # every rank counts its shard's (canonical) k-mers, the spectrum is
        # all-reduced, rank 0 writes it
        src = launch.ShardedSource(engine.default_device(), input_path, k, False)
        try:
            h = src.hist(max_count + 1, canonical=not forward)
        finally:
            src.free()
        if launch.solo_rank():
            with open(output_path, "wb") as fh:
                fh.write(engine.format_hist(h))
        logging.info("That's all!")
        return
    h = engine.abundance_hist(engine.read_input(input_path), k, canonical=not forward, nbins=max_count + 1)
    with open(output_path, "wb") as fh:
        fh.write(engine.format_hist(h))
    logging.info("That's all!")


if __name__ == "__main__":
    main()
