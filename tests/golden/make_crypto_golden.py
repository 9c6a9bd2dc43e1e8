"""Make tests/golden/crypto_fixtures.json: the reference's own encrypted
fixtures, copied as data (base64) so that no test reads /root/reference at
run time.  Run in the build container (where /root/reference exists).

  crates/core/tests/fixtures/{key1,key2,key-failing,config}
      passwords "test" / "test2" (crates/core/tests/keys.rs:12-16)
  crates/core/tests/fixtures/repo-mixed.tar.gz: its key, config, index,
      snapshot and pack file; password "geheim" (tests/integration.rs:113)
"""
import base64
import json
import os
import tarfile

REF = "/root/reference/crates/core/tests/fixtures"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "crypto_fixtures.json")


def b64(b: bytes) -> str:
    return base64.b64encode(b).decode()


def main():
    out = {"source": "rustic_core crates/core/tests/fixtures (copied as data)",
           "keys_test": {}, "repo_mixed": {}}
    for name in ("key1", "key2", "key-failing", "config"):
        out["keys_test"][name] = b64(open(os.path.join(REF, name), "rb").read())
    out["keys_test"]["passwords"] = {"key1": "test", "key2": "test2"}
    t = tarfile.open(os.path.join(REF, "repo-mixed.tar.gz"))
    for m in t.getmembers():
        if m.isfile():
            out["repo_mixed"][m.name] = b64(t.extractfile(m).read())
    out["repo_mixed_password"] = "geheim"
    json.dump(out, open(OUT, "w"), indent=1)
    print(OUT, os.path.getsize(OUT))


if __name__ == "__main__":
    main()
