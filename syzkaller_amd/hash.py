"""Host mirror of hash/hash.go over libsyzgpu.so: Sig = sha1.Sum of a program's text.

    Hash(data) -> Sig                hash.go:13-15
    Sig.String()                     hash.go:17-19  (hex)
    FromString(str) -> Sig           hash.go:21-35
    HashBatch(data, off) -> u8[n,20] the signatures of many programs in one GPU pass (the
                                     persistent-corpus prune, manager.go:541-553; the hub, state.go:209)
"""
from .prog import ProgScan

SIZE = 20  # sha1.Size


class Sig(bytes):
    def String(self):
        return self.hex()

    def __str__(self):
        return self.String()


def HashBatch(data, off=None):
    return ProgScan(data, off, ncalls=False, status=False)[2]


def Hash(data):
    return Sig(bytes(HashBatch([bytes(data)])[0]))


def FromString(s):
    """hash.go:21-35: errors on bad hex or a length other than 20 bytes."""
    try:
        b = bytes.fromhex(s)
    except ValueError as e:
        raise ValueError("failed to decode sig '%s': %s" % (s, e))
    if len(b) != SIZE:
        raise ValueError("failed to decode sig '%s': bad len" % s)
    return Sig(b)


__all__ = ["Sig", "Hash", "HashBatch", "FromString", "SIZE"]
