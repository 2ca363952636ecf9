"""Per-block forward/backward comparison of the HIP Darknet plan against the
oracle (debug helper, not a test)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
import __graft_entry__ as ge
import oracle

cfg, B = sys.argv[1], int(sys.argv[2])
S = int(sys.argv[3]) if len(sys.argv) > 3 else None
dk, W, G, sy = ge._pkg('darknet_v3'), ge._pkg('weights'), ge._pkg('cfg_gen'), ge._pkg('synthetic')
stream = W.synthesize(cfg, seed=4)
path = '/tmp/dbg.weights'
W.write_weights(path, stream)
text = G.cfg_text(cfg)
if S:
    text = text.replace('width=%d' % int(G.cfg_text(cfg).split('width=')[1].split()[0]), 'width=%d' % S).replace(
        'height=%d' % int(G.cfg_text(cfg).split('height=')[1].split()[0]), 'height=%d' % S)
    open('/tmp/dbg.cfg', 'w').write(text)
    cfg = '/tmp/dbg.cfg'
net = dk.Darknet(cfg); net.load_darknet_weights(path)
ref = oracle.OracleDarknet(text, path)
S = ref.height
dev = torch.device('cuda', 0)
x = sy.frames(B, S, seed=7)
# oracle forward keeping every block output
outs = []
xx = x.clone().requires_grad_(True)
h = xx
pre = {}
for i, (d, p) in enumerate(zip(ref.blocks, ref.params)):
    t = d['type']
    if t == 'convolutional':
        h = F.conv2d(h, p['W'], p.get('b'), stride=p['stride'], padding=p['pad'])
        if p['bn']:
            h = F.batch_norm(h, p['bn_rm'], p['bn_rv'], p['bn_w'], p['bn_b'], training=False, eps=1e-5)
        pre[i] = h
        if p['act'] == 'leaky':
            h = F.leaky_relu(h, 0.1)
    elif t == 'maxpool':
        k, s = int(d['size']), int(d['stride'])
        if k == 2 and s == 1: h = F.pad(h, (0, 1, 0, 1))
        h = F.max_pool2d(h, k, s)
    elif t == 'upsample': h = F.interpolate(h, scale_factor=2)
    elif t == 'route': h = torch.cat([outs[int(l)] for l in d['layers'].split(',')], 1)
    elif t == 'shortcut': h = outs[-1] + outs[int(d['from'])]
    h.retain_grad()
    if i in pre: pre[i].retain_grad()
    outs.append(h)
heads_ref = [outs[i] for i, d in enumerate(ref.blocks) if d['type'] == 'yolo']
gen = torch.Generator().manual_seed(9)
grads = [torch.randn(o.shape, generator=gen) for o in heads_ref]
sum((o * g).sum() for o, g in zip(heads_ref, grads)).backward()
xg = x.to(dev).requires_grad_(True)
o = net(xg)
sum((a * g.to(dev)).sum() for a, g in zip(o, grads)).backward()
plan = net.plan(B, S, S, dev)
def rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
for i, d in enumerate(ref.blocks):
    if plan.root[i] != i: continue
    a = plan.act[i].detach().cpu()[..., :plan.shp[i][2]].permute(0, 3, 1, 2)
    fr = rel(a, outs[i].detach())
    gs = ''
    if plan.grad[i] is not None:
        g = plan.grad[i].detach().cpu()[..., :plan.shp[i][2]].permute(0, 3, 1, 2)
        gr = pre[i].grad if (i in pre and plan._leaky(i)) else outs[i].grad
        if gr is not None:
            gs = 'grad rel %.2e' % rel(g, gr)
    print(i, d['type'], plan.shp[i], 'fwd rel %.2e' % fr, gs)
print('dx rel', rel(xg.grad.cpu(), xx.grad))

# ---- isolate the contributions to one block's gradient
if len(sys.argv) > 4:
    tgt = int(sys.argv[4])
    cons = [j for j in range(len(ref.blocks)) if plan.root[j] == j and tgt in plan.srcs[j] and plan.has_grad[j]]
    print('consumers of', tgt, cons)
    import ctypes
    nat = ge._pkg('_native')
    st = nat.stream()
    for j in cons:
        # oracle contribution of consumer j (conv only): conv_transpose of D_j
        dj = pre[j].grad if plan._leaky(j) else outs[j].grad
        Wf, _ = net._folded(j)
        m = net._conv_meta[j]
        contrib = F.conv_transpose2d(dj.double(), Wf, stride=m['stride'], padding=m['pad'],
                                     output_padding=(outs[tgt].shape[-1] - ((dj.shape[-1] - 1) * m['stride'] - 2 * m['pad'] + m['k'])))
        # GPU: run only that consumer's dgrad ops with accumulate=0 and no mask
        descs = plan._dgrad_descs(j, tgt, 0)
        out = torch.zeros_like(plan.grad[tgt])
        for desc, wd in descs:
            nat.call('po_conv', ctypes.byref(desc), nat.ptr(plan.grad[j]), nat.ptr(wd), None, nat.ptr(out), None, None, None, st)
        torch.cuda.synchronize()
        g = out.cpu()[..., :plan.shp[tgt][2]].permute(0, 3, 1, 2).double()
        print('consumer', j, 'D rel', rel(plan.grad[j].cpu()[..., :plan.shp[j][2]].permute(0, 3, 1, 2), dj), 'contrib rel', rel(g, contrib), [ (d.Hg, d.Wg, d.ntaps, d.N, d.Cin_p) for d, _ in descs])
    if len(cons) == 2:
        j1, j2 = cons[1], cons[0]     # processing order: larger j first
        out = torch.zeros_like(plan.grad[tgt])
        for desc, wd in plan._dgrad_descs(j1, tgt, 0):
            nat.call('po_conv', ctypes.byref(desc), nat.ptr(plan.grad[j1]), nat.ptr(wd), None, nat.ptr(out), None, None, None, st)
        torch.cuda.synchronize()
        o1 = out.clone()
        for desc, wd in plan._dgrad_descs(j2, tgt, 1):
            nat.call('po_conv', ctypes.byref(desc), nat.ptr(plan.grad[j2]), nat.ptr(wd), None, nat.ptr(out), None, None, nat.ptr(plan.act[tgt]), st)
        torch.cuda.synchronize()
        g = out.cpu()[..., :plan.shp[tgt][2]].permute(0, 3, 1, 2)
        print('manual seq rel', rel(g, pre[tgt].grad), 'plan G rel', rel(plan.grad[tgt].cpu()[..., :plan.shp[tgt][2]].permute(0, 3, 1, 2), pre[tgt].grad),
              'manual vs plan', rel(out.cpu(), plan.grad[tgt].cpu()))
        # mask-only check
        out2 = o1.clone()
        for desc, wd in plan._dgrad_descs(j2, tgt, 1):
            nat.call('po_conv', ctypes.byref(desc), nat.ptr(plan.grad[j2]), nat.ptr(wd), None, nat.ptr(out2), None, None, None, st)
        torch.cuda.synchronize()
        m = (plan.act[tgt] > 0).float() * 0.9 + 0.1
        print('acc-only then mask rel', rel((out2 * m).cpu()[..., :plan.shp[tgt][2]].permute(0, 3, 1, 2), pre[tgt].grad))
    a = plan.act[tgt].cpu()[..., :plan.shp[tgt][2]].permute(0, 3, 1, 2)
    mm = (a > 0) != (pre[tgt].detach() > 0)
    print('mask mismatches', int(mm.sum()), 'values gpu', a[mm][:8].tolist(), 'oracle pre', pre[tgt].detach()[mm][:8].tolist(),
          'scale', float(pre[tgt].detach().abs().max()))
