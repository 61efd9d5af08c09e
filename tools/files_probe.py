"""Where the file -> file compaction leg's store phase goes (diagnostic):
config-3 inputs through sstc_compact_files with fsync on and off, and the raw
cost of writing + fsyncing the same bytes from host memory with 8 threads.

    python tools/files_probe.py
"""
import os
import sys
import tempfile
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lsm-kv-storage_amd"), ROOT]
import sstcodec  # noqa: E402
from sstcodec import workload as W  # noqa: E402
from sstcodec.table import build_table  # noqa: E402


def main():
    codec = sstcodec.Codec(0)
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        paths, sizes = [], []
        for i, rec in enumerate(W.config_inputs(3, 0)):
            p = os.path.join(td, f"in{i}.sst")
            fs, _ = build_table(codec, p, rec, 4096)
            paths.append(p)
            sizes.append(fs)
        pipe = sstcodec.FilePipe(codec, io_threads=8)
        for fsync in (True, False, True, False):
            od = tempfile.mkdtemp(dir=td)
            t0 = time.perf_counter()
            outs, tm = pipe.compact_files(paths, sizes, od + "/", 1, 4096, 32 << 20, 1, fsync=fsync)
            dt = time.perf_counter() - t0
            print(f"fsync={fsync}: {dt:.4f} s  " + " ".join(f"{k}={v:.4f}" for k, v in tm.items()), flush=True)
        pipe.close()
        # raw: 28 x 43 MB from host memory, 8 writer threads, pwrite + fsync
        buf = np.random.default_rng(0).integers(0, 256, 43_844_060, dtype=np.uint8).tobytes()
        for fsync in (True, False):
            od = tempfile.mkdtemp(dir=td)
            nxt = [0]
            lock = threading.Lock()

            def writer():
                while True:
                    with lock:
                        t = nxt[0]
                        nxt[0] += 1
                    if t >= 28:
                        return
                    fd = os.open(os.path.join(od, f"{t}.sst"), os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
                    os.pwrite(fd, buf, 0)
                    if fsync:
                        os.fsync(fd)
                    os.close(fd)
            t0 = time.perf_counter()
            ths = [threading.Thread(target=writer) for _ in range(8)]
            for th in ths:
                th.start()
            for th in ths:
                th.join()
            print(f"raw 28 x 43.8 MB, 8 threads, fsync={fsync}: {time.perf_counter() - t0:.4f} s", flush=True)


if __name__ == "__main__":
    main()
