import sys, numpy as np, torch
sys.path.insert(0, '.')
from psyne_amd import TDTConfig, TdtCodec
blob = bytes.fromhex('44544454' '00040000' '01000000' '04000000' '04000000') + bytes(16) + (10).to_bytes(4,'little') + bytes([0xff,0]*4+[4,0])
b2 = b'UNCP'[::-1] if False else bytes([0x50,0x43,0x4e,0x55]) + bytes(range(8))
buf = np.frombuffer(blob + b2, np.uint8).copy()
off = np.array([0, len(blob), len(blob)+len(b2)], np.int64)
c = TdtCodec(TDTConfig())
d = torch.from_numpy(buf).cuda(); o = torch.from_numpy(off).cuda()
sizes, st = c.decoded_sizes(d, o)
print('sizes', sizes.cpu().numpy(), 'st', st.cpu().numpy())
out, doff, st2 = c.decode_batch(d, o)
torch.cuda.synchronize()
print('doff', doff.cpu().numpy(), 'st', st2.cpu().numpy(), 'out', out.numel(), out[:8].cpu().numpy())
