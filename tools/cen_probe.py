import os, sys, ctypes
sys.path.insert(0, '/root/repo')
import numpy as np, torch
from tests.test_gpu_fullsize import _c3, NITER
from tests.cases import oracle_pds, rel
pds, case = _c3(torch.float32, 'centered')
est, conv, diag = pds.iterate()
eng = pds._engine
print('engine', type(eng).__name__, 'march', getattr(eng, 'march', None), 'nm_fused', getattr(eng, 'nm_fused', None),
      'path', eng.lib.pcs_pds2d_path(ctypes.byref(eng.args)) if hasattr(eng, 'args') else None, flush=True)
case['tau'], case['sigma'], case['rho'] = pds.tau, pds.sigma, pds.rho
xr, zr, dr = oracle_pds(case, conv_method='fft')
x = est['primal_variable'].double().cpu().numpy(); z = est['dual_variable'].double().cpu().numpy()
print('SPLIT', os.environ.get('PCS_SM_SPLIT'), 'rel x', rel(x, xr), 'rel z', rel(z, zr), flush=True)
