// Operator schemas of the gnnqc HIP library (torch.ops.gnnqc.*).
// Implementations register for the CUDA (= HIP on ROCm) dispatch key in each
// kernel file; CPU callers use the eager PyTorch paths in gnnqc/ops.
#include <ATen/ATen.h>
#include <torch/library.h>

TORCH_LIBRARY(gnnqc, m) {
  // persistent LSTM recurrence (lstm.hip)
  m.def("lstm_fwd(Tensor x, Tensor W, Tensor U, Tensor b, bool train, bool bf16) -> Tensor[]");
  m.def("lstm_bwd(Tensor dh, Tensor gates, Tensor cseq, Tensor U, bool bf16) -> Tensor");
  m.def("lstm_grads(Tensor dz, Tensor x, Tensor hseq, Tensor W, Tensor(a!) dW, Tensor(b!) dU, Tensor(c!) db, "
        "bool need_dx) -> Tensor");
  // fused GeneralConv + BatchNorm + PReLU + node pooling (gcn.hip)
  m.def("gcn_stats(Tensor x, Tensor mask) -> Tensor");
  m.def("gcn_pool_fwd(Tensor x, Tensor w, Tensor anom, Tensor W, Tensor b, Tensor scale, Tensor shift, "
        "Tensor alpha) -> Tensor");
  m.def("gcn_pool_bwd(Tensor x, Tensor w, Tensor dout, Tensor W, Tensor b, Tensor scale, Tensor shift, "
        "Tensor alpha, int c_off) -> Tensor");
  m.def("gcn_pool_bwd_input(Tensor x, Tensor w, Tensor mask, Tensor dout, Tensor W, Tensor b, Tensor scale, "
        "Tensor shift, Tensor alpha, Tensor dzcoef, int c_off) -> Tensor");
  // flat-buffer optimiser (adam.hip)
  m.def("adam_step(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, Tensor lr, Tensor step, float beta1, "
        "float beta2, float eps, float grad_scale, float weight_decay) -> ()");
  m.def("nonfinite_count(Tensor x) -> Tensor");
  // metrics (metrics.hip)
  m.def("score_histogram(Tensor scores, Tensor labels, Tensor mask, int bins) -> Tensor");
  // window gather (gather.hip)
  m.def("window_gather(Tensor series, Tensor shift, Tensor scale, Tensor win_group, Tensor win_center, "
        "Tensor win_valid, Tensor wids, int tb, int seq_len, bool time_norm) -> Tensor");
}
