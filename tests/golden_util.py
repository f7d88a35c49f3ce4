"""Fixture helpers: rebuild generator-spec inputs and compare blobs."""
import hashlib
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def make_input(spec, oracle):
    if "hex" in spec:
        return bytes.fromhex(spec["hex"])
    if "ascii" in spec:
        return spec["ascii"].encode("latin1")
    g = spec["gen"]
    if g == "fill":
        return bytes([spec["byte"]]) * spec["n"]
    if g == "concat":
        return b"".join(make_input(p, oracle) for p in spec["parts"])
    return oracle.gen(g, spec["seed"], spec["n"])


def blob_bytes(b):
    """Bytes of a fixture blob when stored (inline hex or a binary file)."""
    if "hex" in b:
        return bytes.fromhex(b["hex"])
    if "file" in b:
        with open(os.path.join(GOLDEN, b["file"]), "rb") as f:
            return f.read()
    return None


def blob_matches(b, data):
    if len(data) != b["len"]:
        return False
    if "hex" in b:
        return data.hex() == b["hex"]
    return hashlib.sha256(data).hexdigest() == b["sha256"]
