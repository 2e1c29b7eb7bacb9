"""Which kernels run for the separable-PSF deconvolution with a centred K (fused normal-operator
march or the two-launch path): a few iterations of the sep_cen_f32 slab-test problem, single GPU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tests.slab_worker import synth_problem  # noqa: E402


def main():
    torch.cuda.set_device(0)
    pds = synth_problem('sep_cen_f32', niter=6)
    pds.iterate()
    eng = pds._engine
    print('engine', type(eng).__name__, 'march', getattr(eng, 'march', None), 'nm_fused', getattr(eng, 'nm_fused', None),
          'fkind', eng.fkind, 'native', getattr(eng, 'native', None), flush=True)


if __name__ == '__main__':
    main()
