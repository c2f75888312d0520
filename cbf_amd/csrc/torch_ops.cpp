// torch_ops.cpp -- the thin PyTorch-ROCm extension over the C ABI (include/cbf_amd.h).
//
// Registers torch.ops.cbf_amd.* (TORCH_LIBRARY): each op checks its tensors, allocates its outputs
// with the caching allocator and calls the C ABI on the current HIP stream, so the ops compose with
// torch code and can be captured in a hipGraph (torch.cuda.graph).  Host code only: every kernel
// lives in libcbf_amd.so.  Reference surface: ControlBarrierFunction.get_safe_control (cbf.py:18)
// batched, and the callers' per-agent loop (cross_and_rescue.py:135-160) / timestep (:97-175).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <cmath>
#include <tuple>

#include "cbf_amd.h"

namespace {

void* stream() { return (void*)c10::hip::getCurrentHIPStream().stream(); }

void check_rc(int rc, const char* what) {
    TORCH_CHECK(rc != CBF_EINVAL, what, ": invalid argument (CBF_EINVAL)");
    TORCH_CHECK(rc == 0, what, ": HIP error ", rc);
}

// every tensor of a call on the device of its first (the op's stream is that device's)
void check_device(const at::Tensor& ref, const at::Tensor& t, const char* name) {
    TORCH_CHECK(t.device() == ref.device(), name, " must be on ", ref.device(), " (got ", t.device(), ")");
}

// the lattice ops' persistent state: a zero-filled-before-first-use uint8 workspace, and optional
// int64[1024] statistics (None: the statistics-free kernel instantiation the bench times)
uint64_t* check_lattice_state(const at::Tensor& pos, const at::Tensor& workspace,
                              const c10::optional<at::Tensor>& stats) {
    TORCH_CHECK(workspace.is_cuda() && workspace.scalar_type() == at::kByte && workspace.is_contiguous(),
                "workspace must be a contiguous uint8 GPU tensor");
    check_device(pos, workspace, "workspace");
    if (!stats) return nullptr;
    TORCH_CHECK(stats->is_cuda() && stats->scalar_type() == at::kLong && stats->is_contiguous() &&
                    stats->numel() == 1024,
                "stats must be an int64[1024] GPU tensor (or None)");
    check_device(pos, *stats, "stats");
    return reinterpret_cast<uint64_t*>(stats->data_ptr<int64_t>());
}

void check_f64(const at::Tensor& t, const char* name, int64_t cols) {
    TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
    TORCH_CHECK(t.scalar_type() == at::kDouble, name, " must be float64");
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
    TORCH_CHECK(t.dim() == 2 && t.size(1) == cols, name, " must be (n, ", cols, ")");
}

// ControlBarrierFunction(max_speed, dmin, k) with the callers' f = 0 / g = 0.1 [I2; 0] unless given
cbf_params make_params(double max_speed, double dmin, double k, const c10::optional<at::Tensor>& f,
                       const c10::optional<at::Tensor>& g, double safety_distance) {
    cbf_params p;
    at::Tensor fc, gc;
    if (f) {
        fc = f->to(at::kCPU, at::kDouble).contiguous();
        TORCH_CHECK(fc.numel() == 16, "f must be 4 x 4");
    }
    if (g) {
        gc = g->to(at::kCPU, at::kDouble).contiguous();
        TORCH_CHECK(gc.numel() == 8, "g must be 4 x 2");
    }
    check_rc(cbf_params_init(&p, max_speed, dmin, k, f ? fc.data_ptr<double>() : nullptr,
                             g ? gc.data_ptr<double>() : nullptr, safety_distance),
             "cbf_params_init");
    return p;
}

// get_safe_control (cbf.py:18-92) for a batch of egos with CSR neighbour lists.
std::tuple<at::Tensor, at::Tensor> get_safe_control_batch(const at::Tensor& robot_state, const at::Tensor& u0,
                                                          const at::Tensor& nbr_off, const at::Tensor& obs_states,
                                                          double max_speed, double dmin, double k,
                                                          const c10::optional<at::Tensor>& f,
                                                          const c10::optional<at::Tensor>& g) {
    check_f64(robot_state, "robot_state", 4);
    check_f64(u0, "u0", 2);
    check_f64(obs_states, "obs_states", 4);
    const int64_t n = robot_state.size(0);
    TORCH_CHECK(u0.size(0) == n, "u0 must have one row per ego");
    check_device(robot_state, u0, "u0");
    check_device(robot_state, nbr_off, "nbr_off");
    check_device(robot_state, obs_states, "obs_states");
    TORCH_CHECK(nbr_off.is_cuda() && nbr_off.scalar_type() == at::kInt && nbr_off.is_contiguous() &&
                    nbr_off.dim() == 1 && nbr_off.size(0) == n + 1,
                "nbr_off must be an int32 GPU tensor of n + 1 offsets");
    const cbf_params p = make_params(max_speed, dmin, k, f, g, 0.2);
    at::Tensor u = at::empty({n, 2}, robot_state.options());
    at::Tensor status = at::empty({n}, robot_state.options().dtype(at::kInt));
    check_rc(cbf_get_safe_control_batch(&p, (int32_t)n, robot_state.data_ptr<double>(), u0.data_ptr<double>(),
                                        nbr_off.data_ptr<int32_t>(), obs_states.data_ptr<double>(),
                                        u.data_ptr<double>(), status.data_ptr<int32_t>(), nullptr, stream()),
             "cbf_get_safe_control_batch");
    return {u, status};
}

// The per-agent loop of cross_and_rescue.py:135-160 over a swarm (all-pairs cull, LDS-tiled):
// entities [0, n_obs) obstacles, the rest agents (the egos).
std::tuple<at::Tensor, at::Tensor, at::Tensor> filter_swarm(const at::Tensor& pos, const at::Tensor& vel,
                                                            int64_t n_obs, double max_speed, double dmin, double k,
                                                            double safety_distance) {
    check_f64(pos, "pos", 2);
    check_f64(vel, "vel", 2);
    const int64_t n = pos.size(0);
    TORCH_CHECK(vel.size(0) == n && n_obs >= 0 && n_obs <= n, "pos / vel / n_obs do not match");
    check_device(pos, vel, "vel");
    const cbf_params p = make_params(max_speed, dmin, k, c10::nullopt, c10::nullopt, safety_distance);
    const int64_t ne = n - n_obs;
    at::Tensor u = at::empty({ne, 2}, pos.options());
    at::Tensor status = at::empty({ne}, pos.options().dtype(at::kInt));
    at::Tensor cnt = at::empty({ne}, pos.options().dtype(at::kInt));
    if (ne == 0) return {u, status, cnt};
    const size_t need = cbf_allpairs_workspace_size((int32_t)n, (int32_t)ne);
    at::Tensor ws = at::empty({(int64_t)need}, pos.options().dtype(at::kByte));
    check_rc(cbf_filter_allpairs_split(&p, (int32_t)n, (int32_t)n_obs, pos.data_ptr<double>(), vel.data_ptr<double>(),
                                       (int32_t)n_obs, (int32_t)n, u.data_ptr<double>(), status.data_ptr<int32_t>(),
                                       cnt.data_ptr<int32_t>(), ws.data_ptr(), need, stream()),
             "cbf_filter_allpairs_split");
    return {u, status, cnt};
}

// One fused lattice timestep (cbf_lattice_step) of a W x H lattice swarm, positions advanced in
// place.  The cell grid is (x0, y0, cell edge, nx, ny); `workspace` (uint8, zero-filled before its
// first use, cbf_lattice_workspace_size bytes) and `stats` (int64[1024], CBF_STAT_* words, or None
// for the statistics-free kernels) persist across steps; all tensors on pos's device.  Returns (nominal control, filtered control, status, neighbour count).
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> lattice_step(
    at::Tensor pos, int64_t W, int64_t H, double gain, double T, double x0, double y0, double cell, int64_t nx,
    int64_t ny, at::Tensor workspace, c10::optional<at::Tensor> stats, double max_speed, double dmin, double k,
    double safety_distance) {
    check_f64(pos, "pos", 2);
    TORCH_CHECK(pos.size(0) == W * H, "pos must hold W x H agents");
    uint64_t* st = check_lattice_state(pos, workspace, stats);
    const cbf_params p = make_params(max_speed, dmin, k, c10::nullopt, c10::nullopt, safety_distance);
    cbf_grid g;
    g.x0 = x0;
    g.y0 = y0;
    g.inv_h = 1.0 / cell;
    g.nx = (int32_t)nx;
    g.ny = (int32_t)ny;
    const int64_t n = W * H;
    at::Tensor vel = at::empty({n, 2}, pos.options());
    at::Tensor u = at::empty({n, 2}, pos.options());
    at::Tensor status = at::empty({n}, pos.options().dtype(at::kInt));
    at::Tensor cnt = at::empty({n}, pos.options().dtype(at::kInt));
    check_rc(cbf_lattice_step(&p, &g, (int32_t)W, (int32_t)H, 0, (int32_t)H, 0, (int32_t)H, pos.data_ptr<double>(),
                              gain, T, pos.data_ptr<double>(), vel.data_ptr<double>(), u.data_ptr<double>(),
                              status.data_ptr<int32_t>(), cnt.data_ptr<int32_t>(), 0, nullptr,
                              st, workspace.data_ptr(),
                              (size_t)workspace.numel(), stream()),
             "cbf_lattice_step");
    return {vel, u, status, cnt};
}

// `steps` timesteps of the whole lattice in one call (cbf_lattice_run): positions advanced in place,
// bit-identical to `steps` lattice_step calls; returns the last timestep's (nominal control,
// filtered control, status, neighbour count).  window_cull: the lattice-window cull
// (cbf_lattice_run_ex CBF_RUN_WINDOW_CULL), same results.
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> lattice_run(
    at::Tensor pos, int64_t W, int64_t H, double gain, double T, int64_t steps, double x0, double y0, double cell,
    int64_t nx, int64_t ny, at::Tensor workspace, c10::optional<at::Tensor> stats, double max_speed, double dmin, double k,
    double safety_distance, bool window_cull) {
    check_f64(pos, "pos", 2);
    TORCH_CHECK(pos.size(0) == W * H, "pos must hold W x H agents");
    TORCH_CHECK(steps >= 1, "steps must be >= 1 (the outputs are the last timestep's)");
    uint64_t* st = check_lattice_state(pos, workspace, stats);
    const cbf_params p = make_params(max_speed, dmin, k, c10::nullopt, c10::nullopt, safety_distance);
    cbf_grid g;
    g.x0 = x0;
    g.y0 = y0;
    g.inv_h = 1.0 / cell;
    g.nx = (int32_t)nx;
    g.ny = (int32_t)ny;
    const int64_t n = W * H;
    at::Tensor vel = at::empty({n, 2}, pos.options());
    at::Tensor u = at::empty({n, 2}, pos.options());
    at::Tensor status = at::empty({n}, pos.options().dtype(at::kInt));
    at::Tensor cnt = at::empty({n}, pos.options().dtype(at::kInt));
    check_rc(cbf_lattice_run_ex(&p, &g, (int32_t)W, (int32_t)H, pos.data_ptr<double>(), gain, T, (int32_t)steps,
                                vel.data_ptr<double>(), u.data_ptr<double>(), status.data_ptr<int32_t>(),
                                cnt.data_ptr<int32_t>(), st, workspace.data_ptr(), (size_t)workspace.numel(),
                                window_cull ? CBF_RUN_WINDOW_CULL : 0u, stream()),
             "cbf_lattice_run_ex");
    return {vel, u, status, cnt};
}

int64_t lattice_workspace_size(int64_t W, int64_t H, double x0, double y0, double cell, int64_t nx, int64_t ny) {
    cbf_grid g;
    g.x0 = x0;
    g.y0 = y0;
    g.inv_h = 1.0 / cell;
    g.nx = (int32_t)nx;
    g.ny = (int32_t)ny;
    return (int64_t)cbf_lattice_workspace_size((int32_t)W, (int32_t)H, &g);
}

}  // namespace

TORCH_LIBRARY(cbf_amd, m) {
    m.def("get_safe_control_batch(Tensor robot_state, Tensor u0, Tensor nbr_off, Tensor obs_states, float max_speed, "
          "float dmin=0.2, float k=1., Tensor? f=None, Tensor? g=None) -> (Tensor, Tensor)");
    m.def("filter_swarm(Tensor pos, Tensor vel, int n_obs, float max_speed, float dmin=0.2, float k=1., "
          "float safety_distance=0.2) -> (Tensor, Tensor, Tensor)");
    m.def("lattice_step(Tensor(a!) pos, int W, int H, float gain, float T, float x0, float y0, float cell, int nx, "
          "int ny, Tensor(b!) workspace, Tensor(c!)? stats=None, float max_speed=15., float dmin=0.2, "
          "float k=1., float safety_distance=0.2) -> (Tensor, Tensor, Tensor, Tensor)");
    m.def("lattice_run(Tensor(a!) pos, int W, int H, float gain, float T, int steps, float x0, float y0, float cell, "
          "int nx, int ny, Tensor(b!) workspace, Tensor(c!)? stats=None, float max_speed=15., float dmin=0.2, "
          "float k=1., float safety_distance=0.2, bool window_cull=False) -> (Tensor, Tensor, Tensor, Tensor)");
    m.def("lattice_workspace_size(int W, int H, float x0, float y0, float cell, int nx, int ny) -> int",
          &lattice_workspace_size);
    m.def("abi_version() -> int", []() -> int64_t { return cbf_abi_version(); });
}

TORCH_LIBRARY_IMPL(cbf_amd, CUDA, m) {
    m.impl("get_safe_control_batch", get_safe_control_batch);
    m.impl("filter_swarm", filter_swarm);
    m.impl("lattice_step", lattice_step);
    m.impl("lattice_run", lattice_run);
}
