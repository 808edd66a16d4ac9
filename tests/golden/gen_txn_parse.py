#!/usr/bin/env python3
"""Generate tests/golden/txn_parse.npz from the REFERENCE transaction parser
(src/ballet/txn/fd_txn_parse.c compiled in place into oracle/_ref/libfdref_txn.so).

Run in the build container only (needs /root/reference).  Contents:

* ``fix_*``: the reference's own fixtures src/ballet/txn/fixtures/
  transaction{1..6}.bin (data files, stored verbatim) with the reference's
  footprint and full fd_txn_t image for each;
* ``sweep_fp`` / ``sweep_crc``: footprint and CRC-32 of the image for every
  case of tests/txn_builder.sweep_cases (single-byte rewrites of
  transaction1/2/3/6 at every position, as test_txn_parse.c:test_mutate
  does, plus every truncation of all six fixtures);
* ``build_fp`` / ``build_crc``: the same for tests/txn_builder.builder_cases
  (seeded random legacy / v0 transactions with address tables, and
  mutations of them).
"""
from __future__ import annotations

import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle.oracle import RefTxn, build  # noqa: E402
import txn_builder as tb  # noqa: E402

STRIDE = 864


def run(ref, cases):
    arena, off, sz = tb.pack(cases)
    fp, img = ref.txn_parse_batch(arena, off, sz, STRIDE)
    crc = np.array([zlib.crc32(img[i, : fp[i]].tobytes()) for i in range(len(cases))], np.uint32)
    return fp, crc, img


def main() -> None:
    build(ref=True)
    ref = RefTxn()
    fixtures = tb.load_reference_fixtures()
    fa, fo, fs = tb.pack(fixtures)
    ffp, fcrc, fimg = run(ref, fixtures)
    sfp, scrc, _ = run(ref, tb.sweep_cases(fixtures))
    bfp, bcrc, _ = run(ref, tb.builder_cases())
    np.savez_compressed(os.path.join(HERE, "txn_parse.npz"), fix_arena=fa, fix_off=fo, fix_sz=fs, fix_fp=ffp,
                        fix_img=fimg, sweep_fp=sfp, sweep_crc=scrc, build_fp=bfp, build_crc=bcrc)
    print(f"fixtures fp={ffp.tolist()}  sweep {len(sfp)} ({int((sfp > 0).sum())} accepted)  "
          f"builder {len(bfp)} ({int((bfp > 0).sum())} accepted)")


if __name__ == "__main__":
    main()
