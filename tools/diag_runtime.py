import sys, os
sys.path.insert(0, '.')
order = sys.argv[1]
if order == 'torch_first':
    import torch
    print('torch cuda', torch.cuda.is_available(), torch.cuda.device_count())
import my_orb_slam2_amd as m
from my_orb_slam2_amd import synth
L = m.load()
import ctypes
n = ctypes.c_int()
print('devcount rc', L.orbx_device_count(ctypes.byref(n)), n.value, L.orbx_last_error())
try:
    e = m.ORBextractor(2000, 1.2, 8, 20, 7)
    k, d = e(synth.frame(0))
    print('nkp', len(k), k[:3])
except Exception as ex:
    print('ERR', ex)
import subprocess
print(open('/proc/self/maps').read().count('libamdhip64'))
for line in open('/proc/self/maps'):
    if 'libamdhip64' in line or 'hsa-runtime' in line:
        print(line.split()[-1]); 
