"""Write a synthetic .sens of the seeded room in the copyroom / apt0 layout (640x480 JPEG colour, zlib depth,
ground-truth trajectory): BASELINE configs 2 / 3 have no public file here, so their runs use a stream of the
same length and format written on the box (not committed). Usage: python tools/make_sens.py FRAMES PATH"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from bundlefusion_amd.stream import write_synthetic_sens  # noqa: E402

if __name__ == "__main__":
    n, path = int(sys.argv[1]), sys.argv[2]
    w = int(sys.argv[3]) if len(sys.argv) > 3 else 640
    h = int(sys.argv[4]) if len(sys.argv) > 4 else 480
    write_synthetic_sens(path, n, w, h, log=lambda *a: print(*a, flush=True), threads=12)
    print(f"{path}: {os.path.getsize(path) / 1e9:.2f} GB", flush=True)
