#!/usr/bin/env python3
"""Throughput bench: LTE PDSCH transmit path (encode -> rate-match -> scramble -> QAM/RE-map/
precoding -> IDFT + CP) on MI355X, one process per GPU.

Metric (BASELINE.json): DL subframes/s, 20 MHz 2x2 TM3 64-QAM (config C3: MCS 19 on both
codewords, TBS 36696 each, 2 x 14 IDFT-2048 per subframe).  A "step" is one pass of the
transmit path over a batch of --batch synthetic subframes per GPU whose payloads are already
resident in HBM.  Subframes shard across ranks with no data-path collective (weak scaling);
the only collective is the RCCL broadcast of the parameter block from rank 0 (plus the
barriers / max-reduction of the timing harness).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3] [--batch 8192]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def algorithmic_bytes(p, spt):
    """Per subframe: payload read + int16 IQ written; and per kernel."""
    n_cw = p.n_cw
    payload = sum(p.TBS[cw] // 8 for cw in range(n_cw))
    iq = p.nb_antennas_tx * spt * 4
    return payload, iq


def _traffic(config, kernel, batch):
    """Calibrated HBM bytes per launch from the committed rocprofv3 PMC summary
    (tools/summarize_prof.py), only when it was measured at this batch size (else null)."""
    tpath = os.path.join(ROOT, "profiles", f"traffic_{config}.json")
    try:
        t = json.load(open(tpath))
    except Exception:
        return None
    return t.get(kernel) if t.get("batch") == batch else None


def _stage_traffic(config, stage, batch):
    """_traffic of a stage made of several kernels ("k_a+k_b"): the sum, or null if any is missing."""
    parts = [_traffic(config, k, batch) for k in stage.split("+")]
    return None if any(t is None for t in parts) else sum(parts)


def _valu_busy(config, batch):
    """VALU-busy fraction per kernel (SQ_ACTIVE_INST_VALU / CUs / GRBM_GUI_ACTIVE) from the committed
    rocprofv3 --pmc pass (tools/gpu_pmc_valu.sh -> profiles/valu_<config>.json), only when it was
    measured at this batch size (else null)."""
    try:
        t = json.load(open(os.path.join(ROOT, "profiles", f"valu_{config}.json")))
    except Exception:
        return None
    if t.get("batch") != batch:
        return None
    out = {}
    for k, v in t.items():
        if not isinstance(v, dict):
            continue
        name = "encode_rm_scramble" if k.startswith("k_encode") else "modulate_idft_cp" if "k_modofdm" in k else None
        if name:
            out[name] = round(v["valu_busy"], 4)
    return out or None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores():
    """Cores this process may use (the GPU box's CPU share is 16 however many the machine shows)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", "16") or 16), 16))


_PORT_WORKER = r"""
import sys, time, numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + '/tests')
import oracle_lib as O, openair4g_amd as oai
full = sys.argv[6] == "1"
rng = np.random.default_rng(int(sys.argv[5]))
if full:      # --full-grid: subframes 0..9 with CRS + PCFICH/PDCCH (bench.full_grid_items' DCI)
    import bench
    p = oai.make_params(sys.argv[2], subframe=0, subframe_step=1, with_crs=1)
    dci = bench.full_grid_items(p, sys.argv[2])[0]
    cfgs = [O.tx_cfg_from_params(p, sf) for sf in range(10)]
else:
    p = oai.make_params(sys.argv[2], subframe=int(sys.argv[3]))
    dci, cfgs = None, [O.tx_cfg_from_params(p, int(sys.argv[3]))]
pays = [rng.integers(0, 256, size=p.TBS[cw] // 8 + 8, dtype=np.uint8) for cw in range(p.n_cw)]
O.tx_subframe(cfgs[0], pays, dci=dci)
n, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < float(sys.argv[4]):
    O.tx_subframe(cfgs[n % len(cfgs)], pays, dci=dci); n += 1
print(n, time.perf_counter() - t0)
"""


def _port_rate(name, subframe, seconds, procs, full=False):
    """The oracle port in `procs` independent processes for `seconds`: aggregate subframes/s."""
    import subprocess
    ps = [subprocess.Popen([sys.executable, "-c", _PORT_WORKER, ROOT, name, str(subframe), str(seconds), str(i),
                            "1" if full else "0"],
                           stdout=subprocess.PIPE, text=True) for i in range(procs)]
    tot, n_all = 0.0, 0
    for p in ps:
        out, _ = p.communicate()
        n, dt = out.split()
        tot += int(n) / float(dt)
        n_all += int(n)
    return tot, n_all


def _harness_args(p, seconds, seed):
    """argv of oracle/cpu_baseline for an openair4g_amd.TxParams (same configuration)."""
    return [os.path.join(ROOT, "oracle", "cpu_baseline"), f"{seconds}", str(seed), str(p.N_RB_DL),
            str(p.nb_antennas_tx), str(p.mode1_flag), str(p.n_cw), str(p.mimo_mode), str(p.num_pdcch_symbols),
            str(p.first_subframe), str(p.Kmimo), str(p.mcs[0]), str(p.mcs[1] if p.n_cw > 1 else 0), str(p.TBS[0]),
            str(p.TBS[1] if p.n_cw > 1 else 0)] + [hex(p.rb_alloc[i]) for i in range(4)] + [str(p.nb_rb),
                                                                                          str(p.rnti)]


def _harness_rate(p, seconds, procs):
    """oracle/cpu_baseline in `procs` independent processes: (aggregate subframes/s, subframes, the
    per-process JSON lines)."""
    import subprocess
    ps = [subprocess.Popen(_harness_args(p, seconds, 0x5EED + i), stdout=subprocess.PIPE, text=True)
          for i in range(procs)]
    outs = []
    for q in ps:
        out, _ = q.communicate()
        if q.returncode != 0:
            raise RuntimeError(f"oracle/cpu_baseline failed ({q.returncode})")
        outs.append(json.loads(out))
    return sum(o["rate"] for o in outs), sum(o["subframes"] for o in outs), outs


def cpu_baseline(name, seconds, subframe, full=False):
    """The CPU transmit path on the host cores over a bounded sample of the same workload, one core
    and then every core of this process's share (independent processes, as N dlsim instances would
    run).  PDSCH configurations run oracle/cpu_baseline: the reference's own crc24a,
    lte_segmentation, sub_block_interleaving_turbo, lte_rate_matching_turbo, dlsch_scrambling,
    dlsch_modulation (1-2 TX ports) and do_OFDM_mod (-> normal_prefix_mod -> PHY_ofdm_mod ->
    idft2048) compiled unmodified (oracle/_ref), the oracle's restatement where the reference TU
    does not build here (the turbo encoder; the 4-port modulation of C4, which the reference lacks);
    its first subframe is checked bit-exactly against the oracle's whole chain.  The rate is over
    the stages' summed time, as dlsim's phy_proc_tx timer covers them (DCI / pilots excluded).
    `port_share` is the fraction of that time spent in ported stages: the reference's SSE turbo
    encoder may run faster than the scalar port, so the CPU rate is a lower bound on the
    reference's by up to that share.
    --full-grid keeps the oracle port over subframes 0..9 with CRS + PCFICH/PDCCH."""
    import openair4g_amd as oai
    cores = host_cores()
    if full:
        one, n1 = _port_rate(name, subframe, seconds, 1, full)
        allc, nall = _port_rate(name, subframe, max(2.0, seconds / 2), cores, full) if cores > 1 else (one, n1)
        return {"value": one, "unit": "subframes/s", "cores": 1, "kind": "port", "cpu_model": cpu_model(),
                "value_all_cores": allc, "cores_all": cores,
                "sample": f"{n1} subframes of {name} (subframes 0..9 with CRS + PCFICH/PDCCH; the common signals, "
                          f"< 1 % of the REs, not in the CPU sample) through the C oracle on 1 core in {seconds:.0f} s; "
                          f"{nall} on {cores} cores (independent processes)"}
    p = oai.make_params(name, subframe=subframe)
    one, n1, o1 = _harness_rate(p, seconds, 1)
    allc, nall, _ = _harness_rate(p, max(2.0, seconds / 2), cores) if cores > 1 else (one, n1, o1)
    kinds = set(o1[0]["impl"].values())
    return {"value": one, "unit": "subframes/s", "cores": 1,
            "kind": "reference+port" if any(k != "port" for k in kinds) else "port",
            "cpu_model": cpu_model(), "value_all_cores": allc, "cores_all": cores,
            "stage_us_per_subframe": o1[0]["stage_us"], "stage_impl": o1[0]["impl"],
            "port_share": o1[0].get("port_share"),
            "sample": f"{n1} {name} subframes (sf {subframe}) on 1 core in {seconds:.0f} s, {nall} on {cores} cores "
                      f"(independent processes); oracle/cpu_baseline: reference TUs where they build, port "
                      f"elsewhere (stage_impl; port_share of the time in ported stages, which may understate the "
                      f"reference's SSE code there); first subframe bit-exact vs the oracle chain"}


C5_K, C5_CB = 5504, 8          # UL 100 PRB MCS 20: TBS 43816 -> C = 8 blocks of K = 5504
# C5 subframes per step: the decoder runs one wave per 8 code blocks (8 windows each, the reference's
# layout), so 2048 subframes are exactly 2 waves per SIMD and leave the serial recursions' latency
# exposed; throughput rises with the number of rounds a launch holds (k_td16 at 3 waves per SIMD,
# profiles/c5_batch_r05.txt): 2048 -> 236 k, 8192 -> 246 k, 16384 -> 266 k, 24576 -> 275 k,
# 32768 -> 280 k, 49152 -> 283 k subframes/s.  49152 subframes = 393 216 code blocks, 13 GB of LLRs on
# the device, tiled from C5_BASE host rows (c5_llrs, upload_tiled).
C5_BATCH = 49152


C5_BASE = 64                   # distinct code blocks per batch, tiled (no full host copy: ADVICE r05)


def c5_llrs(mode, seed, n=C5_BASE):
    """n distinct decoder inputs (3K+12 int16 each); a batch tiles them (block i = row i % n,
    TurboDecoderBatch.upload_tiled).  "8it" = unstructured LLRs, every CRC check fails, the full 8
    iterations run (SURVEY 8d C5 "8 iterations fixed"); "snr" = CRC-terminated codewords, BPSK
    amplitude 32 + Gaussian noise sigma 28 (early stop)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    if mode == "8it":
        return rng.integers(-40, 41, size=(n, 3 * C5_K + 12), dtype=np.int16)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    import re
    src = open(os.path.join(ROOT, "include", "oai4g_qpp.c")).read()
    f = {int(a): (int(b), int(c)) for a, b, c in re.findall(r"\{\s*(\d+)\s*,\s*(\d+)\s*,\s*(\d+)\s*\}", src)}
    base = []
    for _ in range(n):
        c = np.zeros(C5_K // 8 + 4, dtype=np.uint8)
        c[:(C5_K - 24) // 8] = rng.integers(0, 256, (C5_K - 24) // 8, dtype=np.uint8)
        v = O.crc24b(c, C5_K - 24) >> 8
        c[(C5_K - 24) // 8:(C5_K - 24) // 8 + 3] = [v >> 16, (v >> 8) & 255, v & 255]
        d = O.turbo_encode(c[:C5_K // 8], *f[C5_K]).astype(np.float64)
        base.append(np.clip(np.round((2 * d - 1) * 32 + rng.normal(0, 28, d.size)), -32768, 32767).astype(np.int16))
    return np.stack(base)


C5_TBS, C5_G, C5_QM = 43816, 57600, 4   # UL 100 PRB MCS 20: 12 data symbols x 1200 REs x 16-QAM


def bench_c5_chain(args, world, rank, dist, torch):
    """C5 from the e soft bits (ulsch_decoding.c:1208-1350): per TB of 8 x 5504 blocks, RX rate
    matching + sub-block deinterleaving (k_ul_rm_deint) and the 16-bit decoder (k_td16);
    unstructured soft bits, so every block runs the full 8 iterations."""
    import numpy as np
    import openair4g_amd as oai
    n_sf = args.batch
    rng = np.random.default_rng(0xC5E + rank)
    e = rng.integers(-40, 41, size=(n_sf, C5_G), dtype=np.int16)
    ub = oai.UlDecodeBatch(C5_TBS + 24, C5_G, C5_QM, n_sf, max_iterations=8)
    ub.upload(e)
    sid = torch.cuda.current_stream().cuda_stream
    settle = clock_settle(ub.launch, ub.results, args.settle_ms)
    for _ in range(args.warmup):
        ub.launch()
    ub.results()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ub.launch(stream=sid)
    oai.lib().oai4g_sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    its, _ = ub.results()
    ub.close()
    value = n_sf * args.steps * world / elapsed
    per_launch_ms = elapsed * 1000.0 / args.steps
    alg = n_sf * (2 * C5_G + C5_CB * (C5_K // 8))           # soft bits read + decoded bytes written
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as O
        n, t1 = 0, time.perf_counter()
        while time.perf_counter() - t1 < args.cpu_seconds:
            O.ulsch_decode(e[n % n_sf], C5_TBS + 24, C5_G, C5_QM, max_it=8)
            n += 1
        dt = time.perf_counter() - t1
        cpu = {"value": n / dt, "unit": "subframes/s", "cores": 1, "kind": "port",
               "caveat": "scalar C restatement of the reference's 8-lane SSE decoder (3gpplte_turbo_decoder_sse_16bit.c; its TU needs il_tb/f1f2mat from the missing lte_interleaver.h blob, so it cannot be built here): it may understate the reference CPU by up to ~8x (the SIMD width)", "port_share": 1.0,
               "sample": f"{n} transport blocks (8 x K={C5_K}) through the C oracle chain (RM-rx, deinterleave, "
                         f"decoder16), single thread, {dt:.1f} s"}
    if rank == 0:
        print(json.dumps({
            "metric": "UL subframes/sec (C5 RM-rx + deinterleave + turbo decode)", "value": value,
            "unit": "subframes/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "clock_settle": {"ms": args.settle_ms, "runs": settle, "why": SETTLE_WHY},
            "ms_per_step": per_launch_ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "int16", "data": "synthetic soft bits (unstructured: 8 iterations per block)",
            "config": {"workload": "ulsch_decoding 20 MHz MCS20: G 57600 -> 8 x K=5504, max 8 iterations",
                       "config_id": "C5", "subframes_per_gpu_per_step": n_sf, "mean_iterations": float(np.mean(its)),
                       "parallelism": f"TB-sharded x{world}"},
            "roofline": {"bound": "hbm", "kernel": "k_ul_rm_deint+k_td16", "achieved": alg / (per_launch_ms * 1e-3) / 1e9,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": alg / (per_launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                         "algorithmic_bytes_per_launch": alg},
            "cpu_baseline": cpu}), flush=True)


_C5_WORKER = r"""
import sys, time
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + '/tests')
import bench, oracle_lib as O
llr = bench.c5_llrs(sys.argv[3], 0xC5 + int(sys.argv[5]))
fn = O.turbo_decode8 if sys.argv[2] == "8" else O.turbo_decode
n, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < float(sys.argv[4]):
    fn(llr[n % len(llr)], bench.C5_K, max_it=8, crc_type=1); n += 1
print(n, time.perf_counter() - t0)
"""


def _c5_port_rate(bits, mode, seconds, procs):
    """The oracle decoder in `procs` independent processes: aggregate code blocks/s."""
    import subprocess
    ps = [subprocess.Popen([sys.executable, "-c", _C5_WORKER, ROOT, str(bits), mode, str(seconds), str(i)],
                           stdout=subprocess.PIPE, text=True) for i in range(procs)]
    tot, n_all = 0.0, 0
    for p in ps:
        out, _ = p.communicate()
        n, dt = out.split()
        tot += int(n) / float(dt)
        n_all += int(n)
    return tot, n_all


def _c5_valu(batch):
    """The decoder's VALU-busy fraction from the committed pass (profiles/valu_C5.json) at this batch:
    the build the per-size dispatch runs for 8 blocks per subframe (k_td16_w3 from 98304 blocks)."""
    try:
        t = json.load(open(os.path.join(ROOT, "profiles", "valu_C5.json")))
    except Exception:
        return None
    k = "k_td16_w3" if 8 * batch >= 98304 else "k_td16"
    return round(t[k]["valu_busy"], 4) if t.get("batch") == batch and k in t else None


def bench_c5(args, world, rank, dist, torch):
    """UL turbo decoding throughput (config C5): subframes of 8 code blocks, K = 5504."""
    import numpy as np
    import openair4g_amd as oai
    from openair4g_amd import dist as odist
    oai.init()
    n_sf = args.batch
    n_cb = n_sf * C5_CB
    crc_type = 1                           # C > 1: per-block CRC24_B (ulsch_decoding.c)
    if args.c5_mode == "chain":
        return bench_c5_chain(args, world, rank, dist, torch)
    llr = c5_llrs(args.c5_mode, 0xC5 + rank)
    dec = (oai.TurboDecoder8Batch if args.c5_bits == 8 else oai.TurboDecoderBatch)(C5_K, n_cb)
    dec.upload_tiled(llr)
    settle = clock_settle(lambda: dec.run(max_iterations=8, crc_type=crc_type), dec.results, args.settle_ms)
    for _ in range(args.warmup):
        dec.run(max_iterations=8, crc_type=crc_type)
    dec.results()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dec.run(max_iterations=8, crc_type=crc_type)
    oai.lib().oai4g_sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    its, _ = dec.results()
    dec.close()
    value = n_sf * args.steps * world / elapsed
    per_launch_ms = elapsed * 1000.0 / args.steps
    small = None
    if n_sf != 2048 and rank == 0 and world == 1:
        # the figure at 2048 subframes per launch (2 waves per SIMD, one round), comparable with the
        # rounds before the batch grew: the same kernel on a smaller launch, 5 timed runs
        d2 = (oai.TurboDecoder8Batch if args.c5_bits == 8 else oai.TurboDecoderBatch)(C5_K, 2048 * C5_CB)
        d2.upload_tiled(llr)
        # the upload leaves the GPU idle long enough for its clocks to drop: settle them again first
        clock_settle(lambda: d2.run(max_iterations=8, crc_type=crc_type), d2.results, args.settle_ms)
        d2.run(max_iterations=8, crc_type=crc_type)
        d2.results()
        t2 = time.perf_counter()
        for _ in range(10):
            d2.run(max_iterations=8, crc_type=crc_type)
        oai.lib().oai4g_sync()
        small = {"subframes_per_step": 2048, "value": 2048 * 10 / (time.perf_counter() - t2), "unit": "subframes/s"}
        d2.close()
    alg = n_cb * (2 * (3 * C5_K + 12) + C5_K // 8)          # LLR read + bits written
    ach = alg / (per_launch_ms * 1e-3) / 1e9
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as O
        n, t1 = 0, time.perf_counter()
        dec_fn = O.turbo_decode8 if args.c5_bits == 8 else O.turbo_decode
        while time.perf_counter() - t1 < args.cpu_seconds:
            dec_fn(llr[n % len(llr)], C5_K, max_it=8, crc_type=crc_type)
            n += 1
        dt = time.perf_counter() - t1
        cores = host_cores()
        allc, nall = _c5_port_rate(args.c5_bits, args.c5_mode, max(2.0, args.cpu_seconds / 2), cores) \
            if cores > 1 else (n / dt, n)
        cpu = {"value": n / C5_CB / dt, "unit": "subframes/s", "cores": 1, "kind": "port",
               "caveat": "scalar C restatement of the reference's 8-lane SSE decoder (3gpplte_turbo_decoder_sse_16bit.c; its TU needs il_tb/f1f2mat from the missing lte_interleaver.h blob, so it cannot be built here): it may understate the reference CPU by up to ~8x (the SIMD width)", "port_share": 1.0,
               "cpu_model": cpu_model(), "value_all_cores": allc / C5_CB, "cores_all": cores,
               "sample": f"{n} code blocks (K={C5_K}, mode {args.c5_mode}) through the C oracle decoder, "
                         f"single thread, {dt:.1f} s; {nall} on {cores} cores (independent processes)"}
        if args.c5_bits == 16 and O.ref_td() is not None:
            # the reference's own CPU decoder where it builds: phy_threegpplte_turbo_decoder_scalar
            # (3gpplte_turbo_decoder.c:883, compiled unmodified into oracle/_ref/libref_td.so), same
            # blocks, same iteration cap, CRC24_B (the K = 5504 blocks fit its buffers)
            from ref_cases import QPP
            f1, f2 = QPP[C5_K]
            nr, t2 = 0, time.perf_counter()
            while time.perf_counter() - t2 < max(2.0, args.cpu_seconds / 2):
                O.ref_turbo_decode_scalar(llr[nr % len(llr)], C5_K, f1, f2, max_it=8, crc_type=crc_type)
                nr += 1
            dr = time.perf_counter() - t2
            # the reference's own code is the baseline; the SSE-decoder restatement stays beside it
            port = cpu
            cpu = {"value": nr / C5_CB / dr, "unit": "subframes/s", "cores": 1, "kind": "reference",
                   "sample": f"{nr} code blocks (K={C5_K}, mode {args.c5_mode}) through "
                             f"phy_threegpplte_turbo_decoder_scalar (3gpplte_turbo_decoder.c:883, the reference "
                             f"compiled unmodified), max 8 iterations, single thread, {dr:.1f} s",
                   "caveat": "the reference's scalar decoder; its default 8-lane SSE 16-bit decoder "
                             "(3gpplte_turbo_decoder_sse_16bit.c) needs the missing lte_interleaver.h blob and "
                             "cannot be built here", "port_share": 0.0, "cpu_model": cpu_model(),
                   "sse16_restatement": port}
    if rank == 0:
        print(json.dumps({
            "metric": "UL subframes/sec (C5 turbo decode)" + (", 8-bit decoder" if args.c5_bits == 8 else ""),
            "value": value, "unit": "subframes/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "clock_settle": {"ms": args.settle_ms, "runs": settle, "why": SETTLE_WHY}, "ms_per_step": per_launch_ms, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int8" if args.c5_bits == 8 else "int16",
            "data": f"synthetic LLRs ({args.c5_mode})",
            "config": {"workload": "ulsim 20 MHz MCS20 decode: 8 x K=5504, "
                                   + ("8-bit (16-window)" if args.c5_bits == 8 else "16-bit") + " max-log-MAP, max 8 iterations",
                       "config_id": "C5", "subframes_per_gpu_per_step": n_sf, "code_blocks_per_step": n_cb,
                       "mean_iterations": float(np.mean(its)), "parallelism": f"block-sharded x{world}"},
            "at_2048_subframes": small,
            "roofline": {"bound": "hbm", "kernel": "k_td8" if args.c5_bits == 8 else "k_td16", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS, "traffic": None if args.c5_bits == 8 else _traffic("C5", "k_td16", n_sf),
                         "valu_issue_frac": None if args.c5_bits == 8 or args.c5_mode != "8it" else _c5_valu(n_sf),
                         "note": "latency-bound: traffic (scratch streaming per half-iteration) >> algorithmic bytes"},
            "cpu_baseline": cpu}), flush=True)


_FEP_WORKER = r"""
import sys, time, ctypes, numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + '/tests')
import oracle_lib as O
from test_fep_cpu import window_start
N, n_ant = 2048, int(sys.argv[3])
fpo = O.frame(100, nb_antennas_tx=2, mode1_flag=0)
spt, nsym = fpo.samples_per_tti, fpo.symbols_per_tti
rng = np.random.default_rng(int(sys.argv[4]))
buf = np.zeros(spt + N + 64, np.int32)
frame = buf[(-buf.ctypes.data % 64) // 4:][:spt + N]
frame[:spt] = rng.integers(-2**31, 2**31, size=spt, dtype=np.int64).astype(np.int32)
obuf = np.zeros(nsym * N + 64, np.int32)
rxF = obuf[(-obuf.ctypes.data % 64) // 4:][:nsym * N]
wins = [window_start(fpo, l, Ns, 0, 0) for Ns in (0, 1) for l in range(nsym // 2)]
ref = O.ref_dfts()
fn = ref.dft2048 if ref is not None else (lambda x, y, s: O.orc().orc_dft(11, x, y, s))
n, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < float(sys.argv[2]):
    for a in range(n_ant):
        for i, st in enumerate(wins):
            fn(ctypes.c_void_p(frame.ctypes.data + 4 * st), ctypes.c_void_p(rxF.ctypes.data + 4 * N * i), 1)
    n += 1
print(n, time.perf_counter() - t0)
"""


def _fep_port_rate(seconds, procs, n_ant):
    """slot_fep's dft2048 loop (reference build if present, else the oracle) in `procs` processes."""
    import subprocess
    ps = [subprocess.Popen([sys.executable, "-c", _FEP_WORKER, ROOT, str(seconds), str(n_ant), str(i)],
                           stdout=subprocess.PIPE, text=True) for i in range(procs)]
    tot, n_all = 0.0, 0
    for p in ps:
        out, _ = p.communicate()
        n, dt = out.split()
        tot += int(n) / float(dt)
        n_all += int(n)
    return tot, n_all


def bench_fep(args, world, rank, dist, torch):
    """UE receive front end (SURVEY 8f item 3, config "FEP"): slot_fep of every symbol of
    20 MHz subframes on 2 receive antennas (CP removal + 14 x dft2048 per antenna), batched."""
    import numpy as np
    import openair4g_amd as oai
    oai.init()
    n_sf, n_ant = args.batch, 2
    fp = oai.frame_parms(100, nb_antennas_tx=2, mode1_flag=0)
    N, nsym, spt = fp.ofdm_symbol_size, fp.symbols_per_tti, fp.samples_per_tti
    rng = np.random.default_rng(0xFE9 + rank)
    rx = rng.integers(-3000, 3000, (n_sf, n_ant, 2 * spt), dtype=np.int16).view(np.int32)
    fb = oai.FepBatch(fp, n_sf, n_ant)
    fb.upload(rx)
    settle = clock_settle(fb.run, oai.lib().oai4g_sync, args.settle_ms)
    for _ in range(args.warmup):
        fb.run()
    oai.lib().oai4g_sync()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        fb.run(stream=torch.cuda.current_stream().cuda_stream)
    oai.lib().oai4g_sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # k_fep launch duration for the roofline: HIP events on the launch stream around each launch
    sid = torch.cuda.current_stream().cuda_stream
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.kernel_reps)]
    for e0, e1 in evs:
        e0.record()
        fb.run(stream=sid)
        e1.record()
    torch.cuda.synchronize()
    kern_ms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / len(evs)
    fb.close()
    value = n_sf * args.steps * world / elapsed
    per_launch_ms = elapsed * 1000.0 / args.steps       # one k_fep launch per step
    alg = n_sf * n_ant * nsym * N * 4 * 2                # DFT windows read + frequency symbols written
    ach = alg / (kern_ms * 1e-3) / 1e9
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import ctypes
        import oracle_lib as O
        from test_fep_cpu import window_start
        ref = O.ref_dfts()                               # the reference's own lte_dfts.c (oracle/_ref)
        fpo = O.frame(100, nb_antennas_tx=2, mode1_flag=0)
        buf = np.zeros(spt + N + 64, np.int32)
        frame = buf[(-buf.ctypes.data % 64) // 4:][:spt + N]
        frame[:spt] = rx[0, 0]
        obuf = np.zeros(nsym * N + 64, np.int32)
        rxF = obuf[(-obuf.ctypes.data % 64) // 4:][:nsym * N]
        nsl = nsym // 2
        wins = [window_start(fpo, l, Ns, 0, 0) for Ns in (0, 1) for l in range(nsl)]   # 16-B aligned at 20 MHz
        fn = ref.dft2048 if ref is not None else (lambda x, y, s: O.orc().orc_dft(11, x, y, s))
        n, t1 = 0, time.perf_counter()
        while time.perf_counter() - t1 < args.cpu_seconds:
            for a in range(n_ant):
                for i, st in enumerate(wins):            # slot_fep: dft straight from the rx buffer
                    fn(ctypes.c_void_p(frame.ctypes.data + 4 * st), ctypes.c_void_p(rxF.ctypes.data + 4 * N * i), 1)
            n += 1
        dt = time.perf_counter() - t1
        cores = host_cores()
        allc, nall = _fep_port_rate(max(2.0, args.cpu_seconds / 2), cores, n_ant) if cores > 1 else (n / dt, n)
        cpu = {"value": n / dt, "unit": "subframes/s", "cores": 1, "kind": "reference" if ref is not None else "port",
               "cpu_model": cpu_model(), "value_all_cores": allc, "cores_all": cores,
               "sample": f"{n} subframes x {n_ant} antennas x {nsym} dft2048 ("
                         f"{'the reference lte_dfts.c dft2048 built into oracle/_ref' if ref is not None else 'C oracle'}"
                         f"), single thread, {dt:.1f} s; {nall} on {cores} cores (independent processes)"}
    if rank == 0:
        print(json.dumps({
            "metric": "UE RX front-end subframes/sec (slot_fep, 20 MHz, 2 RX)", "value": value, "unit": "subframes/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "clock_settle": {"ms": args.settle_ms, "runs": settle, "why": SETTLE_WHY}, "ms_per_step": per_launch_ms,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int16",
            "data": "synthetic int16 IQ, resident in HBM",
            "config": {"workload": "slot_fep 20 MHz normal CP, 2 RX antennas, 14 x dft2048 per antenna",
                       "config_id": "FEP", "subframes_per_gpu_per_step": n_sf, "parallelism": f"subframe-sharded x{world}"},
            "roofline": {"bound": "hbm", "kernel": "k_fep<11>", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS, "traffic": _traffic("FEP", "k_fep<11>", n_sf), "kernel_ms": kern_ms,
                         "algorithmic_bytes_per_launch": alg},
            "cpu_baseline": cpu}), flush=True)


def bench_ue(args, world, rank, dist, torch):
    """UE PDSCH receive chain.  Config "UE": dlsim's C2 receiver with
    perfect_ce = 0 -- slot_fep of every symbol, lte_dl_channel_estimation of the pilot symbols
    with the temporal interpolation of every row, rx_pdsch (extraction, channel level,
    compensation, 16-QAM LLRs) and dlsch_unscrambling -- over a batch of consecutive 20 MHz TM1
    subframes (1 TX, 1 RX antenna) produced once by the GPU transmit pipeline.  Config "UE3": the
    C3 receiver (TM3 large-delay CDD, 2 TX x 2 RX, H = I): slot_fep of both antennas, the four
    (port, antenna) estimations, rx_pdsch's TM3 branch (extract_rbs_dual, channel_level_TM3,
    prec2A_TM3 + compensation_TM3, MRC, codeword 0's 64-QAM LLRs) and dlsch_unscrambling."""
    import numpy as np
    import openair4g_amd as oai
    oai.init()
    tm3 = args.config == "UE3"
    n_sf = args.batch
    nrx = 2 if tm3 else 1
    if tm3:
        p = oai.make_params("C3", subframe=0, subframe_step=1, with_crs=1, rnti=0x1234)
        fp = oai.frame_parms(100, nb_antennas_tx=2, mode1_flag=0)
    else:
        p = oai.make_params("C2", subframe=0, subframe_step=1, with_crs=1, rnti=0x1234)
        fp = oai.frame_parms(100)
    N, nsym, spt = fp.ofdm_symbol_size, fp.symbols_per_tti, fp.samples_per_tti
    Qm = oai.lib().oai4g_get_Qm(p.mcs[0])
    # input: n_sf + 1 consecutive transmitted subframes (the last one's symbol 0 closes rows 12 / 13);
    # TM3: receive antenna a = transmit antenna a (H = I)
    tx = oai.TxPipeline(p, n_sf + 1)
    tx.fill_payload(0x5EED + rank)
    tx.run()
    tx.sync()
    fb = oai.FepBatch(fp, n_sf + 1, nrx)
    fb.upload(tx.iq())
    tx.close()
    sid = torch.cuda.current_stream().cuda_stream
    if tm3:
        rb = oai.RxBatchTM3(fp, list(p.rb_alloc), Qm, oai.lib().oai4g_get_Qm(p.mcs[1]), p.mcs[0],
                            p.num_pdcch_symbols, p.rnti, n_sf, nb_rx=2, first_subframe=0)
        cb = None

        if args.ue_unfused:   # the four 14-row estimate planes through memory
            def step(stream):
                fb.run(stream=stream)
                rb.estimate(fb.d_rxF, stream=stream)
                rb.launch(fb.d_rxF, 1, stream=stream)
            stages = {"k_fep": lambda: fb.run(stream=sid), "k_chest x4": lambda: rb.estimate(fb.d_rxF, stream=sid),
                      "k_rx_level_tm3+k_rx_llr_tm3": lambda: rb.launch(fb.d_rxF, 1, stream=sid)}
        else:                 # the 5 pilot rows only; the demodulator interpolates the other rows
            def step(stream):
                fb.run(stream=stream)
                rb.estimate_pilots(fb.d_rxF, stream=stream)
                rb.launch_pilots(fb.d_rxF, 1, stream=stream)
            stages = {"k_fep": lambda: fb.run(stream=sid),
                      "k_chest pilots x4": lambda: rb.estimate_pilots(fb.d_rxF, stream=sid),
                      "k_rx_level_tm3+k_rx_llr_tm3 (pilot rows)": lambda: rb.launch_pilots(fb.d_rxF, 1, stream=sid)}
    else:
        cb = oai.ChestBatch(fp, n_sf, first_subframe=0)
        rb = oai.RxBatch(fp, list(p.rb_alloc), Qm, p.num_pdcch_symbols, p.rnti, n_sf, first_subframe=0,
                         subframe_step=1)

        def step(stream):
            fb.run(stream=stream)
            if args.ue_unfused:
                cb.launch(fb.d_rxF, stream=stream)
                rb.launch(fb.d_rxF, cb.d_est, 1, stream=stream)
            else:
                rb.launch_estimated(cb, fb.d_rxF, 1, stream=stream)
        if args.ue_unfused:
            stages = {"k_fep": lambda: fb.run(stream=sid), "k_chest": lambda: cb.launch(fb.d_rxF, stream=sid),
                      "k_rx_level+k_rx_llr": lambda: rb.launch(fb.d_rxF, cb.d_est, 1, stream=sid)}
        else:
            stages = {"k_fep": lambda: fb.run(stream=sid),
                      "k_rx_chest": lambda: rb.launch_estimated(cb, fb.d_rxF, 1, stream=sid)}
    settle = clock_settle(lambda: step(None), oai.lib().oai4g_sync, args.settle_ms)
    for _ in range(args.warmup):
        step(None)
    oai.lib().oai4g_sync()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(sid)
    oai.lib().oai4g_sync()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # per-stage launch durations (HIP events on the launch stream)
    kern_ms = {}
    for name, fn in stages.items():
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.kernel_reps)]
        for e0, e1 in evs:
            e0.record()
            fn()
            e1.record()
        torch.cuda.synchronize()
        kern_ms[name] = sum(e0.elapsed_time(e1) for e0, e1 in evs) / len(evs)
    n_llr = sum(rb.llr_count(i % 10) for i in range(n_sf))
    n_re = n_llr // Qm
    alg = {"k_fep": (n_sf + 1) * nrx * (spt * 4 + nsym * N * 4),        # IQ read + frequency grid written
           "k_chest": n_sf * (nsym * N * 4 + 5 * N * 4),                   # 14 rows written + 5 pilot rows read
           "k_chest x4": 4 * n_sf * (nsym * N * 4 + 5 * N * 4),
           "k_rx_level+k_rx_llr": n_re * 8 + n_llr * 2 + n_sf * 1200 * 4,  # y + h per RE, LLRs, level row
           "k_rx_chest": n_re * 4 + n_llr * 2 + n_sf * 5 * 1200 * 4,       # y per RE, LLRs, 5 pilot rows
           # 2 y + 4 h per RE, LLRs, the level symbol's 4 estimate rows
           "k_rx_level_tm3+k_rx_llr_tm3": n_re * 24 + n_llr * 2 + n_sf * 4 * 1200 * 4,
           # 4 pilot-row pairs (1216 columns) written, 5 pilot rows of the grid read
           "k_chest pilots x4": 4 * n_sf * (8 * 1216 * 4 + 5 * N * 4),
           "k_rx_level_tm3+k_rx_llr_tm3 (pilot rows)": n_re * 8 + n_llr * 2 + n_sf * 4 * 8 * 1216 * 4}
    alg = {k: v for k, v in alg.items() if k in stages}
    fb.close()
    if cb is not None:
        cb.close()
    rb.close()
    value = n_sf * args.steps * world / elapsed
    dom = max(kern_ms, key=kern_ms.get)
    ach = alg[dom] / (kern_ms[dom] * 1e-3) / 1e9
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = _ue_cpu_baseline(args, p, Qm, tm3)
    if tm3:
        metric = "UE PDSCH RX subframes/sec (20 MHz TM3 2x2 64-QAM, estimated channel)"
        wl = ("slot_fep x2 + lte_dl_channel_estimation (2 ports x 2 RX) + rx_pdsch TM3 (dual extraction, "
              "level_TM3, prec2A/compensation_TM3, MRC, codeword-0 LLRs) + dlsch_unscrambling, C3 20 MHz"
              + (" (14-row estimate planes through memory)" if args.ue_unfused else
                 " (pilot rows only; the demodulator interpolates the estimate rows)"))
    else:
        metric = "UE PDSCH RX subframes/sec (20 MHz TM1 16-QAM, 1 RX, estimated channel)"
        wl = ("slot_fep + lte_dl_channel_estimation + rx_pdsch + dlsch_unscrambling, C2 20 MHz"
              + (" (estimation and demodulation as separate kernels)" if args.ue_unfused else
                 " (estimation fused into the demodulator)"))
    if rank == 0:
        print(json.dumps({
            "metric": metric, "value": value,
            "unit": "subframes/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "clock_settle": {"ms": args.settle_ms, "runs": settle, "why": SETTLE_WHY},
            "ms_per_step": elapsed * 1000.0 / args.steps, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int16",
            "data": f"GPU-transmitted {'C3' if tm3 else 'C2'} subframes (synthetic payload), resident in HBM",
            "config": {"workload": wl, "config_id": args.config, "subframes_per_gpu_per_step": n_sf,
                       "parallelism": f"subframe-sharded x{world}"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS, "traffic": _stage_traffic(args.config, dom, n_sf),
                         "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": alg},
            "end_to_end_algorithmic_GBps": sum(alg.values()) / (elapsed / args.steps) / 1e9,
            "cpu_baseline": cpu}), flush=True)


def _ue_cpu_baseline(args, p, Qm, tm3):
    """The C oracle's UE chain, one thread, on random samples of one subframe (+ the next slot)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    fpo = O.frame(100, nb_antennas_tx=2, mode1_flag=0) if tm3 else O.frame(100)
    N, spt = fpo.ofdm_symbol_size, fpo.samples_per_tti
    nrx = 2 if tm3 else 1
    rng = np.random.default_rng(1)
    frames = []
    for _ in range(nrx):
        f = np.zeros(10 * spt + N, np.int32)
        f[:2 * spt] = rng.integers(-2000, 2000, (2 * spt, 2), dtype=np.int16).view(np.int32).ravel()
        frames.append(f)
    rxF = [np.zeros(15 * N, np.int32) for _ in range(nrx)]
    nxt = [np.zeros(15 * N, np.int32) for _ in range(nrx)]
    n, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < args.cpu_seconds:
        for Ns in (0, 1):
            for l in range(7):
                O.slot_fep(frames, rxF, fpo, l, Ns)
        O.slot_fep(frames, nxt, fpo, 0, 2)
        if tm3:
            est = {(pp, a): O.chest_subframe(fpo, rxF[a][:14 * N], nxt[a][:N], 0, p=pp) for pp in (0, 1)
                   for a in (0, 1)}
            llr, _ = O.rx_pdsch_tm3(fpo, [rxF[0][:14 * N], rxF[1][:14 * N]], est, list(p.rb_alloc), Qm, Qm,
                                    p.mcs[0], p.num_pdcch_symbols, 0)
        else:
            est = O.chest_subframe(fpo, rxF[0][:14 * N], nxt[0][:N], 0)
            llr, _ = O.rx_pdsch_siso(fpo, rxF[0][:14 * N], est, list(p.rb_alloc), Qm, p.num_pdcch_symbols, 0)
        u = np.zeros(32 * (1 + len(llr) // 32), np.int16)
        u[:len(llr)] = llr
        O.dlsch_unscrambling(u, len(llr), (p.rnti << 14) + fpo.Nid_cell)
        n += 1
    dt = time.perf_counter() - t1
    what = ("slot_fep x2 antennas + 4 x 5 lte_dl_channel_estimation calls + rx_pdsch TM3" if tm3 else
            "slot_fep + 5 lte_dl_channel_estimation calls + rx_pdsch")
    return {"value": n / dt, "unit": "subframes/s", "cores": 1, "kind": "port",
            "sample": f"{n} subframes through the C oracle ({what} + dlsch_unscrambling), single thread, {dt:.1f} s"}


SETTLE_WHY = ("GPU power-management ramp: launched cold, the first ~25 ms of back-to-back batches run "
              "~4 % slower than steady state (profiles/clock_settle_r05.txt); the settle runs precede the "
              "warmup steps and are not timed")


def clock_settle(run, sync, ms):
    """Run the step (untimed) until `ms` of wall time has passed, so the timed steps see the GPU's
    steady-state clocks, as a continuously running eNB does; returns the runs made (0 with ms <= 0)."""
    n = 0
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        run()
        n += 1
        if n % 4 == 0:
            sync()
    sync()
    return n


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a launcher: start N fresh child processes of this script, one
    per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT as torch.distributed.run
    sets them), before this process imports torch or touches a GPU.  Rank 0's JSON line reaches
    stdout directly; a failing rank stops the others and the exit code is non-zero."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    live = set(range(n))
    while live:
        for r in sorted(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.discard(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print(f"bench: rank {r} exited with {c}; stopping the other ranks", file=sys.stderr)
                for q in live:
                    procs[q].send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return rc


class Host:
    """Device-side plumbing of the timing harness: RCCL + HIP on the GPU, or (--cpu-stub) gloo on
    the CPU so the rank / broadcast / barrier / max-reduce code runs in the CPU test suite."""

    def __init__(self, args, world, rank, local_rank):
        import torch
        self.torch, self.world, self.rank, self.dist = torch, world, rank, None
        self.local_rank = local_rank
        self.stub = args.cpu_stub
        self.device = "cpu" if self.stub else "cuda"
        if not self.stub:
            torch.cuda.set_device(local_rank)
        if world > 1:
            import torch.distributed as dist
            self.dist = dist
            if self.stub or args.backend == "gloo":
                dist.init_process_group(args.backend)
            else:
                dist.init_process_group(args.backend, device_id=torch.device("cuda", local_rank))

    def sync(self):
        if not self.stub:
            self.torch.cuda.synchronize()

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max_over_ranks(self, v):
        if self.dist is None:
            return v
        t = self.torch.tensor([v], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(self, v):
        if self.dist is None:
            return v
        t = self.torch.tensor([v], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def gather_over_ranks(self, v):
        """Every rank's value, in rank order (an all-gather of one float per rank)."""
        if self.dist is None:
            return [v]
        ts = [self.torch.zeros(1, dtype=self.torch.float64, device=self.device) for _ in range(self.world)]
        self.dist.all_gather(ts, self.torch.tensor([v], dtype=self.torch.float64, device=self.device))
        return [float(t.item()) for t in ts]

    def close(self):
        if not self.stub and self.world > 1:
            import openair4g_amd as oai
            oai.lib().oai4g_dist_finalize()
        if self.dist is not None:
            self.dist.destroy_process_group()


class StubPipeline:
    """CPU stand-in for TxPipeline under --cpu-stub (harness test only: no GPU, no oracle): the
    same methods, a payload-sized XOR fold per subframe as the 'work'."""

    def __init__(self, params, n_sf):
        import numpy as np
        import openair4g_amd as oai
        self.np, self.params, self.n_sf = np, params, n_sf
        self.spt = 30720 if params.N_RB_DL == 100 else 1920
        self.fp = oai.frame_parms(params.N_RB_DL, params.Nid_cell, params.Ncp, params.nb_antennas_tx,
                                  params.mode1_flag, 0)
        self.checksum = 0

    def fill_payload(self, seed):
        rng = self.np.random.default_rng(seed)
        self.pay = rng.integers(0, 2 ** 63, size=(self.n_sf, self.params.payload_stride // 8), dtype=self.np.uint64)

    def run(self, stream=None):
        self.checksum ^= int(self.np.bitwise_xor.reduce(self.pay, axis=None))

    def run_timed(self, stream=None):
        t0 = time.perf_counter()
        self.run()
        t1 = time.perf_counter()
        self.run()
        return (t1 - t0) * 1e3, (time.perf_counter() - t1) * 1e3

    def G(self, cw, subframe):
        import openair4g_amd as oai
        p = self.params
        Qm = oai.lib().oai4g_get_Qm(p.mcs[cw])
        return oai.get_G(self.fp, p.nb_rb, list(p.rb_alloc), Qm, 1, p.num_pdcch_symbols, subframe)

    def sync(self):
        pass

    def close(self):
        pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--settle-ms", type=float, default=250.0,
                    help="untimed runs for this long before the warmup steps (GPU clock ramp); 0 = cold start")
    ap.add_argument("--config", default="C3")
    ap.add_argument("--batch", type=int, default=None,
                    help="subframes per GPU per step (default: C3 8192, C4 1024 = BASELINE config 4's 8192 over "
                         "8 GPUs, FEP 8192, C5 C5_BATCH = 49152); measured on C3: 2048 -> 4.20M, 5120 -> 4.56M, 10240 -> 4.67M "
                         "subframes/s (launch tails amortised)")
    ap.add_argument("--subframe", type=int, default=7)
    ap.add_argument("--full-grid", action="store_true",
                    help="transmit configurations: the eNB's whole grid (PDSCH + CRS + PCFICH/PDCCH + PSS/SSS/PBCH + "
                         "PHICH) over subframe indices 0..9 instead of the PDSCH of --subframe")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-reps", type=int, default=5, help="serial runs timed per kernel for the roofline")
    ap.add_argument("--c5-mode", default="8it", choices=["8it", "snr", "chain"],
                    help="C5 decoder inputs; chain = from the e soft bits through RM-rx + deinterleaving")
    ap.add_argument("--c5-bits", type=int, default=16, choices=[16, 8], help="C5 decoder: 16-bit or 8-bit")
    ap.add_argument("--ue-unfused", action="store_true", help="UE: estimate buffer + separate demodulation kernels")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"], help="nccl = RCCL on ROCm")
    ap.add_argument("--cpu-stub", action="store_true",
                    help="harness test on CPU: gloo, StubPipeline, no GPU (exercises ranks/broadcast/timing)")
    args = ap.parse_args()
    if args.batch is None:
        args.batch = {"C3": 8192, "C4": 1024, "FEP": 8192, "UE": 4096, "UE3": 2048, "C5": C5_BATCH}.get(args.config, 2048)
    if args.cpu_stub:
        args.backend = "gloo"

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)

    host = Host(args, world, rank, local_rank)
    torch, dist = host.torch, host.dist
    if args.config in ("C5", "FEP", "UE", "UE3"):
        if host.stub:
            sys.exit("bench: --cpu-stub covers the transmit configurations only")
        {"C5": bench_c5, "FEP": bench_fep, "UE": bench_ue, "UE3": bench_ue}[args.config](args, world, rank, dist, torch)
        host.close()
        return
    bench_tx(args, world, rank, host)
    host.close()


FULL_GRID_DCI_LEN = {"C1": 23, "C2": 39, "C3": 48, "C4": 48}    # format 1 / 2A (dlsim's DCIs), L = 1
FULL_GRID_PBCH_PDU = (0xA5, 0x3C, 0x0F)


def full_grid_items(params, name):
    """The control and common signals of --full-grid: one UE-specific DCI (dlsim.c's format 1 / 2A,
    aggregation 1, CCE from get_nCCE_offset) for PCFICH + PDCCH, PSS + SSS (subframe indices 0 / 5),
    the PBCH (index 0, frame_mod4 0) and one PHICH per subframe (group 0) — phy_procedures_lte_eNb.c's
    txdataF with with_crs = 1."""
    import ctypes
    import openair4g_amd as oai
    L = oai.lib()
    fp = oai.frame_parms(params.N_RB_DL, Nid_cell=params.Nid_cell, Ncp=params.Ncp,
                         nb_antennas_tx=params.nb_antennas_tx, mode1_flag=params.mode1_flag)
    L.oai4g_init_nCCE_table()
    nCCE = L.oai4g_get_nCCE(params.num_pdcch_symbols, ctypes.byref(fp), 1)
    ncce = L.oai4g_get_nCCE_offset(2, nCCE, 0, params.rnti, 7)
    pdu = bytes(range(0x31, 0x39))
    items = [(FULL_GRID_DCI_LEN[name], 1, ncce, params.rnti, pdu)]
    phich = [] if params.mode1_flag == 1 and params.nb_antennas_tx > 1 else \
        [(sf, 0, sf % 8, sf & 1) for sf in range(10)]
    return items, phich


def full_grid_setup(pipe, params, name):
    items, phich = full_grid_items(params, name)
    pipe.set_control(items)
    pipe.set_common(pss_sss=True, pbch_pdu=FULL_GRID_PBCH_PDU, frame_mod4=0, phich=phich)


def bench_tx(args, world, rank, host):
    """Transmit path (C1-C4): a step = one pass of encode + modulate/IDFT/CP over the batch."""
    import numpy as np
    import openair4g_amd as oai
    from openair4g_amd import dist as odist
    dist = host.dist
    if not host.stub:
        if oai.lib().oai4g_set_device(host.local_rank) != 0:
            raise oai.OAI4GError(oai.lib().oai4g_last_error().decode())
        oai.init()
    # ---- parameter block: built on rank 0, broadcast over RCCL (the only collective): the C ABI's
    # oai4g_dist_broadcast_params on the GPU, torch.distributed (gloo) under --cpu-stub ----
    if args.full_grid:           # the eNB's whole grid over all 10 subframe indices (subframe_step 1)
        p0 = oai.make_params(args.config, subframe=0, subframe_step=1, with_crs=1) if rank == 0 else None
    else:
        p0 = oai.make_params(args.config, subframe=args.subframe) if rank == 0 else None
    if dist is None:
        params = p0
    elif host.stub:
        params = odist.broadcast_params(p0, dist, device=host.device)
    else:
        odist.c_dist_init(rank, world, dist)
        params = odist.c_broadcast_params(p0)

    pipe = (StubPipeline if host.stub else oai.TxPipeline)(params, args.batch)
    if args.full_grid and not host.stub:
        full_grid_setup(pipe, params, args.config)
    # this rank's shard of the global stream of synthetic TBs: global subframes [rank B, (rank + 1) B)
    first, _ = odist.shard_range(world * args.batch, rank, world)
    pipe.fill_payload(seed=odist.global_payload_seed(0x5EED0000, first, params))
    pipe.sync()

    settle = clock_settle(pipe.run, pipe.sync, args.settle_ms if not host.stub else 0)
    for _ in range(args.warmup):
        pipe.run()
    pipe.sync()
    host.sync()

    host.barrier()
    host.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pipe.run()
    pipe.sync()
    host.sync()
    host.barrier()
    elapsed = time.perf_counter() - t0

    # per-kernel launch durations for the roofline: the same batch run serially, HIP events on the
    # launch stream around each kernel (outside the timed region)
    kern = [[], []]
    for _ in range(args.kernel_reps):
        a, b = pipe.run_timed()
        kern[0].append(a)
        kern[1].append(b)
    rank_elapsed = host.gather_over_ranks(elapsed)           # per-rank wall time (readable SCALE lines)
    elapsed = host.max_over_ranks(elapsed)
    units = host.sum_over_ranks(args.batch * args.steps)      # subframes all ranks processed

    value = units / elapsed
    ms_per_step = elapsed * 1000.0 / args.steps

    payload_b, iq_b = algorithmic_bytes(params, pipe.spt)
    sfs = range(10) if args.full_grid else [args.subframe]
    G = [sum(pipe.G(cw, sf) for sf in sfs) / len(sfs) for cw in range(params.n_cw)]      # mean over the batch
    ebits_b = sum((g + 7) / 8 for g in G)
    enc_ms = float(np.median(kern[0]))
    mod_ms = float(np.median(kern[1]))
    per_kernel = {            # bytes = the kernel's own boundary (payload -> e words -> IQ), a diagnostic
        "encode_rm_scramble": {"ms": enc_ms, "bytes": args.batch * (payload_b + ebits_b)},
        "modulate_idft_cp": {"ms": mod_ms, "bytes": args.batch * (ebits_b + iq_b)},
    }
    dom = max(per_kernel, key=lambda k: per_kernel[k]["ms"])
    # roofline.achieved: SURVEY 8(d)'s algorithmic bytes per subframe (payload read + IQ written)
    # x the subframes one launch processes, over the dominant kernel's launch time (HIP events)
    alg_launch = args.batch * (payload_b + iq_b)
    ach = alg_launch / (per_kernel[dom]["ms"] * 1e-3) / 1e9
    ptag = args.config + ("_full" if args.full_grid else "")     # profiles/traffic_<tag>.json
    traffic = _traffic(ptag, dom, args.batch)
    prof_ms = _traffic(ptag + "_ms", dom, args.batch)           # rocprofv3 average of the same command

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.config, args.cpu_seconds, args.subframe, args.full_grid)

    if rank == 0:
        cfgname = {"C1": "dlsim 1.4 MHz SISO QPSK MCS9", "C2": "dlsim 20 MHz SISO 16-QAM MCS16",
                   "C3": "dlsim 20 MHz 2x2 TM3 (LARGE_CDD) 64-QAM MCS19x2CW, 2x14 IDFT-2048",
                   "C4": "20 MHz 4 TX TM3 rank 2 on 4 ports (large-delay CDD, build-defined) 64-QAM MCS19x2CW, "
                         "4x14 IDFT-2048"}[args.config]
        if args.full_grid:
            cfgname += " + full eNB grid (CRS, PCFICH/PDCCH, PSS/SSS/PBCH, PHICH) over subframes 0..9"
        out = {
            "metric": ("DL subframes/sec (20 MHz, 2x2, 64-QAM)" if args.config == "C3" else
                       f"DL subframes/sec ({args.config})") + (" full grid" if args.full_grid else ""),
            "value": value,
            "unit": "subframes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup, "clock_settle": {"ms": args.settle_ms, "runs": settle, "why": SETTLE_WHY},
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int16",
            "data": "synthetic (device-generated splitmix64 transport blocks, resident in HBM)" if not host.stub
                    else "cpu-stub harness run (no GPU): not a measurement",
            "config": {"workload": cfgname, "config_id": args.config, "subframes_per_gpu_per_step": args.batch,
                       "global_batch": args.batch * world,
                       "subframe_index": "0..9 (subframe_step 1)" if args.full_grid else args.subframe,
                       "full_grid": bool(args.full_grid),
                       "TBS": [params.TBS[cw] for cw in range(params.n_cw)], "G": G,
                       "parallelism": f"subframe-sharded x{world}"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
                         "algorithmic_bytes_per_launch": alg_launch,
                         "bytes_basis": f"SURVEY 8(d): payload + IQ = {payload_b + iq_b} B per subframe x "
                                        f"{args.batch} subframes per launch",
                         "timing": f"HIP events around each kernel on its launch stream, median of "
                                   f"{args.kernel_reps} serial runs of the batch (outside the timed region)",
                         "kernel_ms": {k: v["ms"] for k, v in per_kernel.items()},
                         "profiler_ms": prof_ms,
                         "frac_profiler": (alg_launch / (prof_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if prof_ms else None,
                         "valu_issue_frac": _valu_busy(ptag, args.batch),
                         "kernel_boundary_bytes_per_launch": {k: v["bytes"] for k, v in per_kernel.items()},
                         "kernel_boundary_frac": {k: v["bytes"] / (v["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS
                                                  for k, v in per_kernel.items()}},
            "end_to_end_algorithmic_GBps": value * (payload_b + iq_b) / 1e9,
            "per_rank_subframes_per_s": [args.batch * args.steps / e for e in rank_elapsed],
            # value over the sum of the ranks' own rates: 1.0 when every shard takes the same time (the
            # job waits for the slowest); the driver computes scaling efficiency across N itself
            "rank_efficiency": value / sum(args.batch * args.steps / e for e in rank_elapsed),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)

    pipe.close()


if __name__ == "__main__":
    main()
