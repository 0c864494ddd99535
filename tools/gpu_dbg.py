import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["SYZGPU_LIB"] = os.path.join(ROOT, "syzkaller_amd", "libsyzgpu_dbg.so")
from syzkaller_amd import cover
print("start", flush=True)
print("golden minimize", cover.Minimize([[1, 2, 3], [4, 5, 6], [7, 8, 9]]), flush=True)
