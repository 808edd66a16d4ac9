#!/usr/bin/env python3
"""Extract the hex-encoded real transactions of the reference's tile test
(src/disco/verify/test_verify.c:5-106) into tests/golden/verify_tile_txns.json
(data only: the transaction bytes).  Run in the build container only."""
import json
import os
import re

SRC = "/root/reference/src/disco/verify/test_verify.c"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    txt = open(SRC).read()
    out = {"_source": "src/disco/verify/test_verify.c:5-106"}
    for name, body in re.findall(r"static char \*\s*(\w+)\[\] = \{(.*?)\};", txt, flags=re.S):
        body = re.sub(r"//[^\n]*", "", body)
        out[name] = "".join(re.findall(r'"([0-9a-fA-F]*)"', body))
    json.dump(out, open(os.path.join(HERE, "verify_tile_txns.json"), "w"), indent=1)
    print({k: len(v) // 2 for k, v in out.items() if not k.startswith("_")})


if __name__ == "__main__":
    main()
