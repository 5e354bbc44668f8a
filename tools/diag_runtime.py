import os, sys
order = sys.argv[1]
sys.path.insert(0, 'kubernetes-scheduler_amd')
def maps():
    return sorted(set(l.split()[-1] for l in open('/proc/self/maps') if 'amdhip' in l or 'hsa-runtime' in l))
if order == 'torch_first':
    import torch
    print('torch avail', torch.cuda.is_available(), torch.cuda.device_count())
    from yoda_amd.capi import Yoda
    y = Yoda(0); print('yoda ok'); print(maps())
else:
    from yoda_amd.capi import Yoda
    y = Yoda(0); print('yoda ok'); print(maps())
    import torch
    print('torch avail', torch.cuda.is_available(), torch.cuda.device_count())
    print(maps())
print({k: v for k, v in os.environ.items() if 'VISIBLE' in k or 'HIP' in k or 'ROC' in k or 'HSA' in k})
