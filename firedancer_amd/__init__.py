"""firedancer_amd: MI355X-native batch ed25519 signature verification for the
Firedancer verify stage (drop-in for fd_ed25519_verify /
fd_ed25519_verify_batch_single_msg; see include/fd_ed25519_gpu.h)."""
from .engine import (DESC_DTYPE, FD_ED25519_ERR_MSG, FD_ED25519_ERR_PUBKEY, FD_ED25519_ERR_SIG,  # noqa: F401
                     FD_ED25519_SUCCESS, SEMANTICS_AVX512, SEMANTICS_REF, Engine, fd_ed25519_strerror,
                     fd_ed25519_verify, fd_ed25519_verify_batch_single_msg, load_library)
