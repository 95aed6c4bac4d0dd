"""Fixture generator: the calls core.clj makes into the sieve namespace
(alias s/), with their argument counts and lines, read from the reference's
source with tests/clj_reader.py. Output: tests/golden/core_clj_sieve_calls.json
(names, arities and line numbers only -- data, no source text).

  python tests/golden/make_core_calls.py [/root/reference/src/mail_sieve_e/core.clj]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from clj_reader import Form, read_all, walk  # noqa: E402


def sieve_calls(path):
    calls = []
    for f in walk(read_all(open(path).read())):
        if isinstance(f, Form) and f.kind == "(" and f and isinstance(f[0], str) and f[0].startswith("s/"):
            calls.append({"name": f[0][2:], "args": len(f) - 1, "line": f.line})
    return calls


if __name__ == "__main__":
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/src/mail_sieve_e/core.clj"
    out = {"source": "core.clj (dpbriggs/Distributed-Sieve-e src/mail_sieve_e/core.clj)",
           "alias": "[mail-sieve-e.sieve :as s]", "calls": sieve_calls(src),
           "internal": [{"name": "finish", "args": 2, "line": 150, "file": "sieve.clj",
                         "note": "sieve-e's own call, (finish chunk my-num)"}]}
    json.dump(out, open(os.path.join(HERE, "core_clj_sieve_calls.json"), "w"), indent=1)
    print(json.dumps(out["calls"]))
