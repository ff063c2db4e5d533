"""Times the compact hand-over (bfz_record_from_cycles) of the headline record in its parts:
host conversion, the call itself (upload + device rebuild + validation), and the proof, for
rocprofv3 timelines of the events path (`rocprofv3 --kernel-trace --memory-copy-trace -- python3
scripts/events_profile.py`)."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zkvm-brainfuck_amd"))

from bfz import _lib, events, guests, sdk  # noqa: E402

_lib.init(0)
client = sdk.ProverClient()
pk, vk = client.setup(guests.FIBO_X4)
rec = events.ExecutionRecordArrays.from_executor(guests.FIBO_X4, [255])
cyc = events.cycles_from_record(rec)
L = _lib.lib()
for it in range(6):
    t0 = time.perf_counter()
    drec = events.record_from_cycles(pk, cyc, rec.memory)
    t1 = time.perf_counter()
    ptr = ctypes.POINTER(ctypes.c_uint8)()
    plen = ctypes.c_size_t()
    _lib.check(L.bfz_record_prove(ctypes.c_void_p(pk.handle), ctypes.c_void_p(drec.handle),
                                  ctypes.byref(ptr), ctypes.byref(plen), None))
    t2 = time.perf_counter()
    _lib.take_bytes(ptr, plen.value)
    del drec
    print(f"iter {it}: record_from_cycles {1e3 * (t1 - t0):.3f} ms, prove {1e3 * (t2 - t1):.3f} ms",
          flush=True)
