"""``python -m kman_amd count|uniq|batch ...`` — the reference's ``kmer`` CLI."""
from .scripts.kmer import main

main()
