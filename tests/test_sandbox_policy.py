"""The GPU verify tile's and the verify service's seccomp policies (firedancer_amd/
fd_verify_gpu_tile.seccomppolicy, fd_verify_service.seccomppolicy): written in the reference's policy
format (src/disco/verify/fd_verify_tile.seccomppolicy), and allowing every syscall tools/sandbox/
vtile_sandbox measured after privileged_init (profiles/r03/sandbox; round 6, the tile at the bench's
paced defaults with and without its launch thread and the served form: profiles/r06/sandbox): the runs
under those lists completed with every frag published.  The served tile process runs under the reference
verify tile's own two syscalls."""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
POLICY = os.path.join(ROOT, "firedancer_amd", "fd_verify_gpu_tile.seccomppolicy")
SVC_POLICY = os.path.join(ROOT, "firedancer_amd", "fd_verify_service.seccomppolicy")
REF_TILE = ["write", "fsync"]          # src/disco/verify/fd_verify_tile.seccomppolicy


def policy_syscalls(path=POLICY):
    names, params = [], []
    for line in open(path):
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


def _jsonl(path):
    return [json.loads(l) for l in open(path) if l.strip()]


def test_policy_matches_the_measurement():
    names, _ = policy_syscalls()
    for rnd, legs in (("r03", ["discover"]), ("r06", ["discover", "discover_launcher"])):
        d = os.path.join(ROOT, "profiles", rnd, "sandbox")
        for leg in legs:
            disc = json.load(open(os.path.join(d, leg + ".json")))
            enf = json.load(open(os.path.join(d, leg.replace("discover", "enforce") + ".json")))
            # every syscall the tile made after init is allowed; the enforced run published every frag
            assert set(disc["syscalls_after_init"]) <= set(names), (rnd, leg)
            assert enf["rc"] == 0 and enf["published"] == enf["frags"] and not enf["syscalls_after_init"]
    r06 = os.path.join(ROOT, "profiles", "r06", "sandbox")
    assert [json.load(open(os.path.join(r06, f)))["launcher"] for f in ("enforce.json", "enforce_launcher.json")] \
        == [0, 1]


def test_service_policy_and_served_tile():
    """The served form: the tile process makes no syscall after init and has no GPU descriptor, so it runs
    under the reference verify tile's own policy; its service runs under fd_verify_service.seccomppolicy."""
    names, params = policy_syscalls(SVC_POLICY)
    assert names == ["write", "fsync", "ioctl", "futex", "exit_group"]
    assert params == ["logfile_fd", "kfd_fd", "drm_fd"]
    d = os.path.join(ROOT, "profiles", "r06", "sandbox")
    disc = {r["role"]: r for r in _jsonl(os.path.join(d, "served_discover.json"))}
    enf = {r["role"]: r for r in _jsonl(os.path.join(d, "served_enforce.json"))}
    tile, svc = disc["tile"], disc["service"]
    assert set(tile["syscalls_after_init"]) <= set(REF_TILE) and tile["gpu_open"] == 0 and tile["driver_fds"] == 0
    assert set(svc["syscalls_after_init"]) <= set(names)
    for r in enf.values():
        assert r["rc"] == 0 and r["published"] == r["frags"] and not r["syscalls_after_init"]
    assert enf["service"]["completed"] == enf["service"]["frags"]
    assert enf["tile"]["gpu_open"] == 0
    # the enforce leg ran with exactly these lists (tools/gpu_sandbox.sh records them)
    rec = open(os.path.join(d, "policy_names.txt")).read()
    assert "service policy: " + " ".join(names) in rec
