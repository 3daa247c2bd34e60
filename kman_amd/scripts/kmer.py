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

from .. import __version__
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


def _batches(input_path, k, reverse, scan_mode, batch_size, batch_mode, threads, tmp):
    return (
        FastaBatcher(scan_mode=FastaBatcher.MODE[scan_mode], reverse=reverse, size=batch_size, threads=threads,
                     tmp=tmp)
        .do(input_path, k, BatcherThreading.FEED_MODE[batch_mode])
        .collection
    )


@main.command(name="count", context_settings=CONTEXT_SETTINGS, help="""
Count occurrences of all k-mers from INPUT.

\b
Counting modes:
       SEQ_COUNT a tabulation-separated table with sequence and count
       VEC_COUNT / VEC_COUNT_MASKED: abundance vectors (not supported; the
                 reference raises NotImplementedError for them as well)
The INPUT file can be gzipped.
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
    if previous_batches is not None:
        batches = load_batches(previous_batches, threads, re_sort)
    else:
        batches = _batches(input_path, k, reverse, scan_mode, batch_size, batch_mode, threads, tmp)
    prep_joiner(KJoinerThreading(KJoiner.MODE[count_mode], KJoiner.MEMORY[memory_mode]), len(batches),
                threads).join(batches, output_path)
    logging.info("That's all!")


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
    if previous_batches is not None:
        batches = load_batches(previous_batches, threads, re_sort)
    else:
        batches = _batches(input_path, k, reverse, scan_mode, batch_size, batch_mode, threads, tmp)
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
    if os.path.isdir(output_path) and len(os.listdir(output_path)) != 0:
        raise AssertionError("output folder must be empty or non-existent.")
    set_tempdir(tmp)
    os.makedirs(output_path, exist_ok=True)
    try:
        copy_batches(_batches(input_path, k, reverse, scan_mode, batch_size, batch_mode, threads, tmp),
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
    from .. import engine

    input_file_exists(input_path)
    h = engine.abundance_hist(engine.read_input(input_path), k, canonical=not forward, nbins=max_count + 1)
    with open(output_path, "wb") as fh:
        fh.write(engine.format_hist(h))
    logging.info("That's all!")


if __name__ == "__main__":
    main()
