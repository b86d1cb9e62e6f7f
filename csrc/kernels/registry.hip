// Operator schemas of the gnnqc HIP library (torch.ops.gnnqc.*).
// Implementations register for the CUDA (= HIP on ROCm) dispatch key in each
// kernel file; CPU callers use the eager PyTorch paths in gnnqc/ops.
#include <ATen/ATen.h>
#include <torch/library.h>

#include "common.h"

namespace gq {
bool lstm_defer_reduce(bool flag);      // lstm_tm.hip
int64_t lstm_reduce_flush();
// returns the previous value (see deterministic_mode in common.h)
static bool set_deterministic(bool flag) {
  const bool old = deterministic_mode();
  deterministic_mode() = flag;
  return old;
}
}  // namespace gq

TORCH_LIBRARY(gnnqc, m) {
  // process-wide switches (catch-all kernels: no tensor arguments)
  m.def("set_deterministic(bool flag) -> bool", &gq::set_deterministic);
  m.def("lstm_defer_reduce(bool flag) -> bool", &gq::lstm_defer_reduce);
  m.def("lstm_reduce_flush() -> int", &gq::lstm_reduce_flush);
  // persistent LSTM recurrence (lstm.hip)
  m.def("lstm_fwd(Tensor x, Tensor W, Tensor U, Tensor b, bool train, bool bf16) -> Tensor[]");
  m.def("lstm_bwd(Tensor dh, Tensor gates, Tensor cseq, Tensor U, bool bf16) -> Tensor");
  m.def("lstm_grads(Tensor dz, Tensor x, Tensor hseq, Tensor W, Tensor(a!) dW, Tensor(b!) dU, Tensor(c!) db, "
        "bool need_dx) -> Tensor");
  // time-major LSTM with fused backward (lstm_tm.hip)
  m.def("lstm_tm_fwd(Tensor x, Tensor W, Tensor U, Tensor b, bool train, bool store_gates=True) -> Tensor[]");
  m.def("lstm_tm2_fwd(Tensor x, Tensor WA, Tensor UA, Tensor bA, Tensor WB, Tensor UB, Tensor bB, "
        "bool train, bool store_gates=True, int pool=0) -> Tensor[]");
  m.def("lstm_tm_grads(Tensor dz, Tensor x, Tensor h, Tensor W, Tensor(a!) dW, Tensor(b!) dU, Tensor(c!) db, "
        "bool need_dx) -> Tensor");
  m.def("lstm_dx(Tensor dz, Tensor W, Tensor like) -> Tensor");
  m.def("lstm_chain_fwd(Tensor x, Tensor[] W, Tensor[] U, Tensor[] b, int[] pool, bool train) -> Tensor[]");
  m.def("lstm_chain_fwd_pack(Tensor x, Tensor[] W, Tensor[] U, Tensor[] b, int[] pool, bool train, Tensor Wt4, "
        "Tensor Ut4) -> Tensor[]");
  m.def("lstm_chain_head_fwd(Tensor x, Tensor[] W, Tensor[] U, Tensor[] b, int[] pool, bool train, Tensor Wt4, "
        "Tensor Ut4, Tensor bt4, Tensor[] head, Tensor y, Tensor mask, int M, float alpha1, float alpha2, float w0, "
        "float w1, Tensor(a!) sums, Tensor(b!) hist) -> Tensor[]");
  m.def("lstm_chain_status(Tensor like) -> Tensor");
  m.def("lstm_chain_capacity(Tensor like) -> int");
  m.def("lstm_chain_ctl(Tensor like) -> Tensor");
  m.def("lstm_grads_multi(Tensor[] gz, Tensor[] gx, Tensor[] gh, Tensor[] gW, int[] period, int[] hshift, "
        "Tensor[] gws, Tensor[] rws, Tensor[] rW, Tensor(a!)[] rdW, Tensor(b!)[] rdU, Tensor(c!)[] rdb, "
        "Tensor[] gcn_t, int[] gcn_i) -> ()");
  m.def("lstm_chain_trace(Tensor like) -> Tensor");
  m.def("lstm_chain_prof(Tensor like) -> Tensor");
  m.def("lstm_chain_bwd(Tensor dh, Tensor[] g, Tensor[] c, Tensor[] W, Tensor[] U, Tensor[] pidx, int[] pool, "
        "int[] x_width, int[] T_in) -> Tensor[]");
  m.def("lstm_chain_head_bwd(Tensor dloss, Tensor x4, Tensor h4, Tensor g4, Tensor c4, Tensor Wt4, Tensor Ut4, "
        "Tensor pk, Tensor hb, Tensor[] head, Tensor y, Tensor mask, int M, float alpha1, float alpha2, float w0, float w1, "
        "Tensor(a!)[] hgrads, Tensor[] g, Tensor[] c, Tensor[] W, Tensor[] U, Tensor[] pidx, int[] pool, "
        "int[] x_width, int[] T_in) -> Tensor[]");
  m.def("time4_head_fwd(Tensor x, Tensor W, Tensor U, Tensor b, Tensor pk, bool train, Tensor[] head, Tensor y, Tensor mask, "
        "int M, float alpha1, float alpha2, float w0, float w1, Tensor(a!) sums, Tensor(b!) hist) -> Tensor[]");
  m.def("time4_head_bwd(Tensor dloss, Tensor x, Tensor h, Tensor g, Tensor c, Tensor W, Tensor U, Tensor pk, Tensor[] head, "
        "Tensor y, Tensor mask, int M, float alpha1, float alpha2, float w0, float w1, Tensor(a!)[] hgrads) -> Tensor[]");
  m.def("time4_trace(Tensor like) -> Tensor");
  m.def("time4_fwd(Tensor x, Tensor W, Tensor U, Tensor b, bool train, bool all_h, int max_blocks=0) -> Tensor[]");
  m.def("time4_bwd(Tensor dh, Tensor x, Tensor g, Tensor c, Tensor W, Tensor U, bool need_dz, int max_blocks=0, "
        "Tensor? row_scale=None) -> Tensor[]");
  m.def("time4_prob_fwd(Tensor x, Tensor W, Tensor U, Tensor b, Tensor[] head, float alpha1, float alpha2, int M, "
        "bool train, int max_blocks=0) -> Tensor[]");
  m.def("lstm_tm_bwd_pipe(Tensor dh, Tensor g, Tensor c, Tensor W, Tensor U, int T, Tensor gz, Tensor gx, "
        "Tensor gh, Tensor gW, int g_period, int g_hshift, Tensor gws, Tensor rws, Tensor rW, Tensor(a!) rdW, "
        "Tensor(b!) rdU, Tensor(c!) rdb) -> Tensor");
  m.def("lstm_grads_job_ws(Tensor dz, Tensor x, Tensor W, int H) -> Tensor");
  m.def("lstm_tm_bwd(Tensor dh, Tensor g, Tensor c, Tensor x, Tensor h, Tensor W, Tensor U, Tensor b, Tensor(a!) dW, "
        "Tensor(b!) dU, Tensor(c!) db, bool need_dx, Tensor? pidx=None, int pool=0) -> Tensor");
  // fused GeneralConv + BatchNorm + PReLU + node pooling (gcn.hip)
  m.def("gcn_stats(Tensor x, Tensor mask) -> Tensor");
  m.def("gcn_pool_fwd(Tensor x, Tensor w, Tensor anom, Tensor W, Tensor b, Tensor scale, Tensor shift, "
        "Tensor alpha, int Mp=0, int Cp=0) -> Tensor");
  m.def("gcn_pool_bwd(Tensor x, Tensor w, Tensor dout, Tensor W, Tensor b, Tensor scale, Tensor shift, "
        "Tensor alpha, int c_off, bool time_major=False) -> Tensor");
  m.def("gcn_pool_bwd_input(Tensor x, Tensor w, Tensor mask, Tensor dout, Tensor W, Tensor b, Tensor scale, "
        "Tensor shift, Tensor alpha, Tensor dzcoef, int c_off, bool time_major=False) -> Tensor");
  // window gather + GeneralConv + pooling from the resident store (gcn_fused.hip)
  m.def("gcn_window_prep(Tensor series, Tensor shift, Tensor scale, Tensor win_group, Tensor win_center, "
        "Tensor win_valid, Tensor group_adj, Tensor group_anom_pos, int tb, int seq_len, bool time_norm, "
        "bool agg_mean, int pool) -> Tensor[]");
  m.def("gcn_fused_fwd(Tensor series, Tensor shift, Tensor scale, Tensor win_group, Tensor win_center, "
        "Tensor win_valid, Tensor win_label, Tensor group_anom_pos, Tensor mom, Tensor pw, Tensor wids, "
        "Tensor table, Tensor? cursor, int tb, int seq_len, bool time_norm, Tensor W, Tensor b, Tensor gamma, "
        "Tensor beta, Tensor alpha, Tensor(a!) rmean, Tensor(b!) rvar, bool training, float momentum, float eps, "
        "int Mp, int Cp, bool with_coef=False, bool defer=False) -> Tensor[]");
  m.def("gcn_fused_bwd(Tensor dh, int c_off, Tensor series, Tensor shift, Tensor scale, Tensor win_group, "
        "Tensor win_center, Tensor win_valid, Tensor group_anom_pos, Tensor pw, Tensor wids, Tensor table, "
        "Tensor? cursor, int tb, int seq_len, bool time_norm, Tensor S, Tensor st, Tensor W, Tensor b, "
        "Tensor alpha, Tensor(a!) dW, Tensor(b!) dgamma, Tensor(c!) dbeta, Tensor(d!) dalpha) -> ()");
  m.def("gcn_coef_flush(Tensor like) -> bool");
  m.def("gcn_prod_flush(Tensor like) -> bool");
  m.def("gcn_coef_bwd(Tensor dh, int c_off, Tensor coef, Tensor S, Tensor st, Tensor W, Tensor b, Tensor(a!) dW, "
        "Tensor(b!) dgamma, Tensor(c!) dbeta, Tensor(d!) dalpha) -> ()");
  // per-node GeneralConv writing the time-major LSTM input (gcn_node.hip)
  m.def("gcn_adj_bits(Tensor adj, bool agg_mean) -> Tensor[]");
  m.def("gcn_node_fwd(Tensor x, Tensor bits, Tensor rs, Tensor mask, Tensor W, Tensor b, Tensor scale, "
        "Tensor shift, Tensor alpha, int Mp, int Cp) -> Tensor");
  m.def("gcn_node_bwd(Tensor x, Tensor bitsT, Tensor rs, Tensor mask, Tensor dout, Tensor W, Tensor b, "
        "Tensor scale, Tensor shift, Tensor alpha) -> Tensor");
  m.def("gcn_node_bwd_input(Tensor x, Tensor bitsT, Tensor rs, Tensor mask, Tensor dout, Tensor W, Tensor b, "
        "Tensor scale, Tensor shift, Tensor alpha, Tensor coef) -> Tensor");
  // GCN glue: pooling weights, BN statistics, closed-form backward (gcn_glue.hip)
  m.def("gcn_pool_weights(Tensor adj, Tensor mask, Tensor anom_pos, bool agg_mean, int pool) -> Tensor");
  m.def("gcn_bn_prep(Tensor S, Tensor W, Tensor b, Tensor gamma, Tensor beta, Tensor(a!) rmean, Tensor(b!) rvar, "
        "bool training, float momentum, float eps) -> Tensor");
  m.def("gcn_prep(Tensor x, Tensor adj, Tensor mask, Tensor anom_pos, bool agg_mean, int pool, Tensor W, Tensor b, "
        "Tensor gamma, Tensor beta, Tensor(a!) rmean, Tensor(b!) rvar, bool training, float momentum, float eps) -> Tensor[]");
  m.def("gcn_bwd_finalize(Tensor acc, Tensor S, Tensor W, Tensor b, Tensor st, bool training, Tensor(a!) dW, "
        "Tensor(b!) db, Tensor(c!) dgamma, Tensor(d!) dbeta, Tensor(e!) dalpha) -> Tensor");
  // Conv1D + LeakyReLU (+ GAP) implicit GEMM (conv1d.hip)
  m.def("conv1d_fwd(Tensor x, Tensor W, Tensor b, float alpha, bool gap, bool store_y) -> Tensor[]");
  m.def("conv1d_bwd(Tensor dy, Tensor y, Tensor x, Tensor W, float alpha, bool gap, Tensor(a!) dW, "
        "Tensor(b!) db, bool need_dx) -> Tensor");
  // flat-buffer optimiser (adam.hip)
  m.def("adam_step(Tensor(a!) p, Tensor(d!) g, Tensor(b!) m, Tensor(c!) v, Tensor lr, Tensor step, float beta1, "
        "float beta2, float eps, float grad_scale, float weight_decay, Tensor? guard=None, bool zero_grad=False) -> ()");
  m.def("adam_guarded(Tensor(a!) p, Tensor(d!) g, Tensor(b!) m, Tensor(c!) v, Tensor lr, Tensor(e!) step, float beta1, "
        "float beta2, float eps, float grad_scale, float weight_decay, Tensor(f!) state, Tensor(g!)? ext=None, "
        "Tensor(h!)? cursor=None, int cursor_mod=1) -> bool");
  m.def("adam_flagged(Tensor(a!) p, Tensor(d!) g, Tensor(b!) m, Tensor(c!) v, Tensor lr, Tensor(e!) step, float beta1, "
        "float beta2, float eps, float grad_scale, float weight_decay, Tensor(f!) state, Tensor(g!) ext, "
        "Tensor(h!)? cursor=None, int cursor_mod=1) -> ()");
  m.def("nonfinite_count(Tensor x) -> Tensor");
  m.def("ig_interp(Tensor v, Tensor alpha) -> Tensor");
  m.def("ig_gcn_pool_fwd(Tensor x, Tensor w, Tensor anom, Tensor W, Tensor b, Tensor scale, Tensor shift, "
        "Tensor alpha, Tensor alphas, int Cp) -> Tensor");
  m.def("ig_gcn_pool_bwd(Tensor x, Tensor w, Tensor mask, Tensor g, Tensor W, Tensor b, Tensor scale, Tensor shift, "
        "Tensor alpha, Tensor alphas, Tensor wts, Tensor(a!) acc_x, Tensor(b!) acc_a, bool overwrite=False) -> ()");
  m.def("ig_accum(Tensor(a!) acc, Tensor g, Tensor w) -> ()");
  m.def("ig_finalize(Tensor acc, Tensor v, int mode) -> Tensor");
  m.def("chain_poison(Tensor(a!) g, Tensor ext) -> ()");
  m.def("grad_guard(Tensor g, Tensor(a!) state, Tensor(b!) step, Tensor(c!)? ext=None) -> ()");
  // metrics (metrics.hip)
  m.def("score_histogram(Tensor scores, Tensor labels, Tensor mask, int bins) -> Tensor");
  // fused dense head + weighted BCE + metrics (head.hip)
  m.def("head_fwd(Tensor feat, Tensor W1, Tensor b1, Tensor W2, Tensor b2, Tensor W3, Tensor b3, Tensor y, "
        "Tensor mask, float alpha1, float alpha2, float w0, float w1, Tensor(a!) sums, Tensor(b!) hist) -> Tensor[]");
  m.def("head_bwd(Tensor feat, Tensor W1, Tensor W2, Tensor W3, Tensor z1, Tensor z2, Tensor logits, Tensor y, "
        "Tensor mask, float alpha1, float alpha2, float w0, float w1, Tensor gout, Tensor aux, Tensor(a!) dW1, "
        "Tensor(b!) db1, Tensor(c!) dW2, Tensor(d!) db2, Tensor(e!) dW3, Tensor(f!) db3, bool need_dfeat) -> Tensor");
  m.def("head_prob_fwd(Tensor feat, Tensor W1, Tensor b1, Tensor W2, Tensor b2, Tensor W3, Tensor b3, float alpha1, "
        "float alpha2) -> Tensor[]");
  m.def("head_prob_bwd(Tensor feat, Tensor W1, Tensor W2, Tensor W3, Tensor z1, Tensor z2, Tensor prob, "
        "float alpha1, float alpha2) -> Tensor");
  // MaxPooling1D with byte argmax (pool.hip)
  m.def("maxpool1d_fwd(Tensor x, int p) -> Tensor[]");
  m.def("maxpool1d_bwd(Tensor dy, Tensor idx, int T, int p) -> Tensor");
  // window gather (gather.hip)
  m.def("window_gather(Tensor series, Tensor shift, Tensor scale, Tensor win_group, Tensor win_center, "
        "Tensor win_valid, Tensor wids, int tb, int seq_len, bool time_norm) -> Tensor");
  m.def("batch_meta(Tensor wids, Tensor win_group, Tensor win_valid, Tensor group_adj, Tensor group_anom_pos, "
        "Tensor win_label, Tensor win_label_valid, Tensor valid_sample, Tensor x) -> Tensor[]");
  m.def("batch_gather(Tensor series, Tensor shift, Tensor scale, Tensor win_group, Tensor win_center, "
        "Tensor win_valid, Tensor wids, Tensor table, Tensor? cursor, Tensor group_adj, Tensor group_anom_pos, "
        "Tensor win_label, Tensor win_label_valid, Tensor valid_sample, int tb, int seq_len, bool time_norm) -> Tensor[]");
}
