"""Writes the C++ source of gs_kernel_hash(): the sha256 prefix (16 hex digits) of the
device sources named on the command line (csrc/*.hip, csrc/*.h), hashed as
gossip_sim_amd.source_hash() hashes them (file name, NUL, contents; by file name)."""
import hashlib
import os
import sys

h = hashlib.sha256()
for f in sorted(sys.argv[1:], key=os.path.basename):
    h.update(os.path.basename(f).encode() + b"\0")
    with open(f, "rb") as fh:
        h.update(fh.read())
print('extern "C" const char* gs_kernel_hash(void) { return "%s"; }' % h.hexdigest()[:16])
