"""Expected results of the raw-payload path (device fd_txn_parse + verify),
computed by the oracle: fd_txn_parse restated, then
fd_ed25519_verify_batch_single_msg over the parsed offsets exactly as
fd_txn_verify slices them (src/disco/verify/fd_verify_tile.h:67-77)."""
import numpy as np

from firedancer_amd.engine import DESC_DTYPE, FDGPU_ERR_PARSE, TXN_IMG_STRIDE


def parsed_desc(fp, img, off, sz):
    """DESC records for the accepted payloads (oracle convention: sig_base = prefix of sig_cnt)."""
    ok = np.nonzero(fp)[0]
    d = np.zeros(len(ok), DESC_DTYPE)
    im = img[ok].astype(np.uint32)
    d["payload_off"] = off[ok]
    d["payload_sz"] = sz[ok]
    d["sig_cnt"] = im[:, 1]
    d["signature_off"] = im[:, 2] | im[:, 3] << 8
    d["message_off"] = im[:, 4] | im[:, 5] << 8
    d["acct_addr_off"] = im[:, 10] | im[:, 11] << 8
    cnt = im[:, 1].astype(np.int64)
    d["sig_base"] = np.concatenate([[0], np.cumsum(cnt)[:-1]]) if len(ok) else []
    return ok, d, int(cnt.sum())


def expected_codes(oracle, arena, off, sz, sem=0, threads=16):
    fp, img = oracle.txn_parse_batch(arena, off, sz, TXN_IMG_STRIDE)
    codes = np.full(len(off), FDGPU_ERR_PARSE, np.int8)
    ok, d, nsig = parsed_desc(fp, img, off, sz)
    if len(ok):
        t, _ = oracle.verify_txns(arena, d, nsig, sem=sem, threads=threads)
        codes[ok] = t
    return codes, fp, img
