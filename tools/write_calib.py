"""WRITE_SIZE calibration for 4-byte words (tests/cpp/spt_testhooks.hip write_calib_kernel):
run under rocprofv3 --pmc WRITE_SIZE; each pattern writes 512 MiB of u32 words 3 times.
Usage (GPU box): rocprofv3 --pmc WRITE_SIZE -d DIR -o run --output-format csv -- python3 tools/write_calib.py"""
import ctypes
import os

import torch

lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "simplepathtracer_amd", "lib")
h = ctypes.CDLL(os.path.join(lib, "libspt_testhooks.so"))
h.spt_test_write_calib.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
words = 128 << 20
buf = torch.zeros(words, dtype=torch.int32, device="cuda")
for pattern in (0, 1):
    for _ in range(3):
        assert h.spt_test_write_calib(None, buf.data_ptr(), words, pattern) == 0
    torch.cuda.synchronize()
    assert int(buf[12345].item()) == 12345
print(f"wrote {words * 4 / 1e6:.1f} MB per launch", flush=True)
