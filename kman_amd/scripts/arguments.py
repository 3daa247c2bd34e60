"""Click arguments/options of the ``kmer`` CLI — same names, short flags and
defaults as the reference (kmermaid/scripts/arguments.py:14-221)."""

from __future__ import annotations

import tempfile

import click

from ..batcher import BatcherThreading, FastaBatcher
from ..join import KJoiner


def input_path():
    return click.argument("input_path", metavar="INPUT",
                          type=click.Path(exists=True, file_okay=True, readable=True))


def output_path(file_okay=False, dir_okay=False):
    return click.argument("output_path", metavar="OUTPUT",
                          type=click.Path(exists=False, file_okay=file_okay, dir_okay=dir_okay, writable=True))


def k():
    return click.argument("k", type=click.INT)


def reverse():
    return click.option("--reverse", "-r", is_flag=True, help="Include also reverse-complemented sequences")


def scan_mode():
    return click.option("--scan-mode", "-s", type=click.Choice([m.name for m in FastaBatcher.MODE],
                                                                case_sensitive=True),
                        default=FastaBatcher.MODE.KMERS.name,
                        help="KMERS: batch the k-mer stream; RECORDS: batch each record. Default: KMERS")


def batch_size():
    return click.option("--batch-size", "-b", type=click.INT, default=1000000,
                        help="Number of k-mers per batch. Default: 1000000")


def batch_mode():
    return click.option("--batch-mode", "-m", type=click.Choice([m.name for m in BatcherThreading.FEED_MODE],
                                                                 case_sensitive=True),
                        default=BatcherThreading.FEED_MODE.APPEND.name,
                        help="How batches are fed to the collection. Default: APPEND")


def previous_batches():
    return click.option("--previous-batches", "-B", type=click.Path(exists=True, dir_okay=True, readable=True),
                        help="Path to folder with previously generated batches.")


def count_mode():
    return click.option("--count-mode", "-m",
                        type=click.Choice([m.name for m in KJoiner.MODE if "COUNT" in m.name], case_sensitive=True),
                        default=KJoiner.MODE.SEQ_COUNT.name, help='Default: "%s"' % KJoiner.MODE.SEQ_COUNT.name)


def memory_mode():
    return click.option("--memory-mode", "-M", type=click.Choice([m.name for m in KJoiner.MEMORY],
                                                                  case_sensitive=True),
                        default=KJoiner.MEMORY.NORMAL.name, help='Default: "%s"' % KJoiner.MEMORY.NORMAL.name)


def threads():
    return click.option("--threads", "-t", type=click.INT, default=1,
                        help="Accepted for compatibility; the GPU path ignores it.")


def tmp():
    return click.option("--tmp", "-T", type=click.Path(exists=True), default=tempfile.gettempdir(),
                        help='Temporary folder path. Default: "%s"' % tempfile.gettempdir())


def compress():
    return click.option("--compress", "-C", is_flag=True, help="Compress output files.")


def re_sort():
    return click.option("--re-sort", "-R", is_flag=True, help="Force batch re-sorting, when loaded with -B.")
