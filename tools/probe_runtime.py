"""Which HIP runtime(s) end up mapped when torch and libgelly_cc share a process, in each load order."""
import ctypes
import subprocess
import sys

LIB = "gelly-streaming_amd/lib/libgelly_cc.so"
CODE = {
    "torch_first": "import torch; a=torch.cuda.is_available(); import ctypes; l=ctypes.CDLL('%s'); n=ctypes.c_int(); l.gcc_device_count(ctypes.byref(n)); b=torch.cuda.is_available()" % LIB,
    "lib_first": "import ctypes; l=ctypes.CDLL('%s'); n=ctypes.c_int(); l.gcc_device_count(ctypes.byref(n)); import torch; a=b=torch.cuda.is_available()" % LIB,
}
for name, code in CODE.items():
    code += ("\nmaps=[x.split()[-1] for x in open('/proc/self/maps') if 'amdhip64' in x or 'hsa-runtime' in x]"
             "\nprint('%s', 'torch_ok', a, b, 'lib_devices', n.value, sorted(set(maps)))" % name)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180)
    print(r.stdout.strip(), r.stderr.strip()[-300:])
