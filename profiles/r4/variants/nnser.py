# every lane's network evaluations on one shared stream (towers never overlap
# each other; the lanes' tree kernels still overlap the towers)
s = open("az_engine.hip").read()
def rep(old, new):
    global s
    assert s.count(old) == 1, old
    s = s.replace(old, new)
rep("""  hipEvent_t move_done[4] = {nullptr, nullptr, nullptr, nullptr};  // end of move m on this lane, m mod 4""",
"""  hipEvent_t move_done[4] = {nullptr, nullptr, nullptr, nullptr};  // end of move m on this lane, m mod 4
  hipEvent_t ev_sel = nullptr, ev_nn = nullptr;""")
rep("""  hipStream_t pack_stream = nullptr;
  bool own_pack_stream = false;""", """  hipStream_t pack_stream = nullptr;
  bool own_pack_stream = false;
  hipStream_t nn_stream = nullptr;""")
rep("""  if (e->cfg.evaluator == AZ_EVAL_NETWORK) {
    // the stem reads the queued boards straight (no encode pass; bitwise the same outputs)
    az::launch_forward(e->net, L.x, n_rows, L.n, L.g.H, L.g.W, L.g.A, L.act[0], L.act[1], L.act[2],
                       L.probs, L.values, s, L.timer.enabled ? &L.timer : nullptr, rows);""",
"""  if (e->cfg.evaluator == AZ_EVAL_NETWORK) {
    hipStream_t ns = s;
    if (e->nn_stream && L.ev_sel) {
      AZ_HIP(hipEventRecord(L.ev_sel, s));
      AZ_HIP(hipStreamWaitEvent(e->nn_stream, L.ev_sel, 0));
      ns = e->nn_stream;
    }
    // the stem reads the queued boards straight (no encode pass; bitwise the same outputs)
    az::launch_forward(e->net, L.x, n_rows, L.n, L.g.H, L.g.W, L.g.A, L.act[0], L.act[1], L.act[2],
                       L.probs, L.values, ns, L.timer.enabled ? &L.timer : nullptr, rows);
    if (ns != s) {
      AZ_HIP(hipEventRecord(L.ev_nn, ns));
      AZ_HIP(hipStreamWaitEvent(s, L.ev_nn, 0));
    }""")
rep("""      for (hipEvent_t& ev : L->move_done)
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
          return cleanup(fail(AZ_E_HIP, "hipEventCreate failed"));
    }
  }""", """      for (hipEvent_t& ev : L->move_done)
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
          return cleanup(fail(AZ_E_HIP, "hipEventCreate failed"));
      if (hipEventCreateWithFlags(&L->ev_sel, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&L->ev_nn, hipEventDisableTiming) != hipSuccess)
        return cleanup(fail(AZ_E_HIP, "hipEventCreate failed"));
    }
    if (hipStreamCreateWithFlags(&e->nn_stream, hipStreamNonBlocking) != hipSuccess)
      return cleanup(fail(AZ_E_HIP, "hipStreamCreate failed"));
  }""")
rep("""  for (Lane* L : eng->lanes) {
    for (hipEvent_t ev : L->move_done)
      if (ev) (void)hipEventDestroy(ev);""", """  if (eng->nn_stream) {
    (void)hipStreamSynchronize(eng->nn_stream);
    (void)hipStreamDestroy(eng->nn_stream);
  }
  for (Lane* L : eng->lanes) {
    for (hipEvent_t ev : L->move_done)
      if (ev) (void)hipEventDestroy(ev);
    if (L->ev_sel) (void)hipEventDestroy(L->ev_sel);
    if (L->ev_nn) (void)hipEventDestroy(L->ev_nn);""")
open("az_engine.hip", "w").write(s)
