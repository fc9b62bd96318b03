import sys, os, tempfile
sys.path[:0] = ['/root/repo', '/root/repo/mdanalysis-mpi_amd', '/root/repo/tests']
import numpy as np, torch
from test_xtc_gpu import _cases, _records, _host_decode
from rmsf_amd._lib import call
from rmsf_amd.xtc import write_xtc
for case, (x, prec) in sorted(_cases().items()):
    p = tempfile.mktemp(suffix='.xtc'); write_xtc(p, x, precision=prec)
    words, off, ln, n_atoms = _records(p)
    ref, hst = _host_decode(words, off, ln, n_atoms)
    dev = torch.device('cuda')
    dw = torch.as_tensor(words.view(np.int32)).to(dev); do = torch.as_tensor(off).to(dev); dl = torch.as_tensor(ln).to(dev)
    out = torch.empty((len(off), n_atoms, 3), dtype=torch.float32, device=dev); st = torch.full((len(off),), -1, dtype=torch.int32, device=dev)
    call('rmsf_xtc_decode_records', dw.data_ptr(), do.data_ptr(), dl.data_ptr(), len(off), n_atoms, out.data_ptr(), 3 * n_atoms, st.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    bad = np.argwhere(o != ref)
    print(case, 'n_atoms', n_atoms, 'host', hst.tolist(), 'dev', st.cpu().tolist(), 'mismatch', len(bad), bad[:3].tolist(), flush=True)
