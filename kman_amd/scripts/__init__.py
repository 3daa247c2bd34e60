"""The ``kmer`` CLI (batch / count / uniq)."""
