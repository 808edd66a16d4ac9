"""The GPU verify tile's seccomp policy (firedancer_amd/fd_verify_gpu_tile.seccomppolicy): written in the
reference's policy format (src/disco/verify/fd_verify_tile.seccomppolicy), and listing exactly the
syscalls tools/sandbox/vtile_sandbox measured after privileged_init (profiles/r03/sandbox): the run under
that list completed with every frag published."""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
POLICY = os.path.join(ROOT, "firedancer_amd", "fd_verify_gpu_tile.seccomppolicy")


def policy_syscalls():
    names, params = [], []
    for line in open(POLICY):
        if line.startswith("#") or not line.strip():
            continue
        if line.startswith("unsigned int"):
            params += [p.strip().split()[-1] for p in line[len("unsigned int"):].split(",")]
            continue
        m = re.match(r"^([a-z_0-9]+)\s*(:|$)", line)
        if m:
            names.append(m.group(1))
    return names, params


def test_policy_format_and_contents():
    names, params = policy_syscalls()
    # the reference tile's two, plus what the HIP runtime needs after init
    assert names == ["write", "fsync", "ioctl", "futex", "exit_group"]
    assert params == ["logfile_fd", "kfd_fd", "drm_fd"]
    text = open(POLICY).read()
    assert re.search(r"ioctl: \(or \(eq \(arg 0\) kfd_fd\)\s+\(eq \(arg 0\) drm_fd\)\)", text)


def test_policy_matches_the_measurement():
    d = os.path.join(ROOT, "profiles", "r03", "sandbox")
    disc = json.load(open(os.path.join(d, "discover.json")))
    enf = json.load(open(os.path.join(d, "enforce.json")))
    names, _ = policy_syscalls()
    # every syscall the tile made after init is allowed; the enforced run published every frag
    assert set(disc["syscalls_after_init"]) <= set(names)
    assert enf["rc"] == 0 and enf["published"] == enf["frags"]
