"""Print every op of the lowered program (no GPU): index, kind, ksize/stride, sources, cout, out HxW,
K steps, n tiles, and the per-launch bytes a conv_fast wave set pulls through the vector memory
path for a given plan (used to check the per-CU load-bandwidth model against measured times)."""
import importlib, json, sys
sys.path.insert(0, ".")
PKG = "yolo---small-target-recognition---kalman-trajectory-prediction_amd"
A = importlib.import_module(PKG + ".arch")
M = importlib.import_module(PKG + ".model")
Wt = importlib.import_module(PKG + ".weights")
ar = A.parse_arch(A.load_model_dict("yolov8s-small.yaml"))
sd = Wt.synthetic_state_dict(ar, 0)
prog = M.Program(ar, sd, 512, 640, 640, 8, "bf16", 300)
ops_t = {}
if len(sys.argv) > 1:
    ops_t = {o["op"]: o for o in json.load(open(sys.argv[1]))["ops"]}
B = 8
for i, op in enumerate(prog.ops):
    if op.kind != M.YK_K_CONV if hasattr(M, "YK_K_CONV") else False:
        print(i, "kind", op.kind)
        continue
    cin = sum(op.src_ch[j] for j in range(op.n_src))
    px = B * op.out_h * op.out_w
    t = ops_t.get(i, {})
    print(i, f"k{op.ksize}s{op.stride}", f"cin {cin:4d} cout {op.cout:4d} out {op.out_h}x{op.out_w} ksteps {op.k_steps} ntiles {op.n_tiles} px {px}",
          t.get("kernel", "")[22:50], t.get("us", ""))
