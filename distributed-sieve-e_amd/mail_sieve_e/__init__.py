"""mail_sieve_e -- MI355X-native drop-in for the hot path of dpbriggs/Distributed-Sieve-e.

Mirrors the reference namespaces:
  mail-sieve-e.sieve (src/mail_sieve_e/sieve.clj) -> mail_sieve_e.sieve
  mail-sieve-e.core  (src/mail_sieve_e/core.clj)  -> mail_sieve_e.core
Compute runs in libdse.so (gfx950 HIP kernels + RCCL); see include/dse.h.
"""
from . import _dse  # noqa: F401
from .sieve import (Chunk, Context, finish, gen_table, sieve_e, spread_work,  # noqa: F401
                    tail_range)

__all__ = ["Chunk", "Context", "finish", "gen_table", "sieve_e", "spread_work", "tail_range"]
