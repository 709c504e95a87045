// Chain compiler: parse -> fuse pointwise runs -> passes with halo/margin contracts.
#include "stripe/chain.h"

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdlib>
#include <sstream>

namespace stripe {

uint8_t PointwiseProgram::apply_channel_lut(uint8_t v) const {
  if (has_pre) v = pre[v];
  if (has_post) v = post[v];
  return v;
}

GrayParams gray_params(GrayMode m) {
  GrayParams gp;
  if (m == GrayMode::Ref) {
    gp.mode = 1;
    const double w[3] = {0.3, 0.59, 0.11};  // R, G, B (kernel.cu:40-42)
    for (int c = 0; c < 3; ++c) {
      bool ok = find_trunc_magic(w[c], &gp.mult[c], &gp.shift[c]);
      STRIPE_CHECK(ok, "no exact integer form for trunc(x*" << w[c] << ")");
    }
  } else {
    gp.mode = 0;
    gp.mult[0] = 4899;
    gp.mult[1] = 9617;
    gp.mult[2] = 1868;
    gp.shift[0] = gp.shift[1] = gp.shift[2] = 14;
  }
  return gp;
}

namespace {

std::array<uint8_t, 256> identity_lut() {
  std::array<uint8_t, 256> l{};
  for (int i = 0; i < 256; ++i) l[i] = (uint8_t)i;
  return l;
}

// Fold a per-channel LUT op into `prog` at its current position.
void fold_lut(PointwiseProgram& prog, const Op& op) {
  if (!prog.gray) {
    if (!prog.has_pre) {
      prog.pre = identity_lut();
      prog.has_pre = true;
    }
    for (auto& v : prog.pre) v = apply_pointwise_u8(op, v);
  } else {
    if (!prog.has_post) {
      prog.post = identity_lut();
      prog.has_post = true;
    }
    for (auto& v : prog.post) v = apply_pointwise_u8(op, v);
  }
}

// Without a gray stage pre and post are one per-channel LUT: keep it in `post`.
void normalize(PointwiseProgram& prog) {
  if (!prog.gray && prog.has_pre) {
    std::array<uint8_t, 256> l{};
    for (int i = 0; i < 256; ++i) l[i] = prog.has_post ? prog.post[prog.pre[i]] : prog.pre[i];
    prog.post = l;
    prog.has_post = true;
    prog.has_pre = false;
  }
  auto is_id = [](const std::array<uint8_t, 256>& l) {
    for (int i = 0; i < 256; ++i)
      if (l[i] != i) return false;
    return true;
  };
  if (prog.has_post && is_id(prog.post)) prog.has_post = false;
  if (prog.has_pre && is_id(prog.pre)) prog.has_pre = false;
}

std::string prog_desc(const PointwiseProgram& p) {
  std::string s;
  if (p.has_pre) s += "lut,";
  if (p.gray) s += p.gmode == GrayMode::Ref ? "gray:ref," : "gray:bt601,";
  if (p.has_post) s += "lut,";
  if (p.expand) s += "expand,";
  if (!s.empty()) s.pop_back();
  return s;
}

}  // namespace

std::string Plan::describe() const {
  std::ostringstream os;
  os << "chain '" << spec << "': " << cin << "ch -> " << cout << "ch, " << passes.size()
     << " pass(es), max radius " << max_radius << "\n";
  for (size_t i = 0; i < passes.size(); ++i) os << "  pass " << i << ": " << passes[i].desc << "\n";
  return os.str();
}

Plan compile_chain(const std::vector<Op>& ops, int cin, Border default_border, bool fuse) {
  STRIPE_CHECK(cin == 1 || cin == 3, "input must have 1 or 3 channels, got " << cin);
  Plan plan;
  plan.spec = chain_to_string(ops);
  plan.cin = cin;
  int c = cin;
  PointwiseProgram pending;
  int pending_cin = c;

  auto flush_pointwise = [&]() {
    normalize(pending);
    if (!pending.identity()) {
      Pass p;
      p.kind = PassKind::Pointwise;
      p.cin = pending_cin;
      p.cout = pending.channels_out(pending_cin);
      p.cmid = p.cout;
      p.pro = pending;
      p.desc = "pointwise[" + prog_desc(pending) + "] " + std::to_string(p.cin) + "->" +
               std::to_string(p.cout) + "ch";
      plan.passes.push_back(p);
    }
    pending = PointwiseProgram{};
    pending_cin = c;
  };

  for (const Op& op : ops) {
    if (op.pointwise()) {
      switch (op.kind) {
        case OpKind::Gray:
          if (c == 1) break;  // gray of gray is the identity
          if (pending.expand || (!fuse && !pending.identity())) flush_pointwise();
          pending.gray = true;
          pending.gmode = op.gray;
          c = 1;
          break;
        case OpKind::Expand:
          STRIPE_CHECK(c == 1, "expand needs a 1-channel image (after gray)");
          if (!fuse && !pending.identity()) flush_pointwise();
          pending.expand = true;
          c = 3;
          break;
        default:
          // a LUT after expand equals the same LUT before it (channels are copies)
          if (!fuse && !pending.identity()) flush_pointwise();
          fold_lut(pending, op);
          break;
      }
      continue;
    }
    // stencil / conv
    Pass p;
    p.border = op.has_border ? op.border : default_border;
    normalize(pending);
    const bool conv = op.kind == OpKind::Conv;
    if (conv || !fuse || !pending.prologue_ok()) flush_pointwise();
    if (conv) {
      STRIPE_CHECK(p.border != Border::Skip, "skip border is only defined for integer stencils");
      p.kind = PassKind::Conv;
      p.K = op.K;
      p.R = op.K / 2;
      p.conv_w = op.weights;
      p.conv_digits = op.conv_digits;
      p.sep_h = op.sep_h;
      p.sep_v = op.sep_v;
      p.cin = p.cmid = p.cout = c;
      p.desc = "conv" + std::to_string(op.K) + "x" + std::to_string(op.K) +
               (p.sep_h.empty() ? (op.K <= 5 || (op.K == 7 && c == 1) ? "(direct) " : "(mfma) ") : "(mfma-separable) ") +
               std::to_string(c) + "ch border=" + border_name(p.border) + (op.conv_digits == 2 ? " lsb" : "");
    } else {
      const StencilInfo& si = stencil_info(op.sid);
      p.kind = si.separable ? PassKind::Separable : PassKind::Direct;
      p.sid = op.sid;
      p.K = si.K;
      p.R = si.K / 2;
      p.cin = pending_cin;
      p.pro = pending;
      p.cmid = p.cout = c;
      std::string pro = prog_desc(pending);
      p.desc = std::string(si.separable ? "separable " : "direct ") + si.name +
               (pro.empty() ? "" : " prologue[" + pro + "]") + " " + std::to_string(p.cin) +
               "->" + std::to_string(p.cout) + "ch border=" + border_name(p.border);
    }
    plan.passes.push_back(p);
    pending = PointwiseProgram{};
    pending_cin = c;
  }
  // trailing pointwise ops: epilogue of the last stencil if they are a LUT and/or
  // an expand of its 1-channel result (the reference's gray -> emboss -> expand
  // GPU chain, kernel.cu:192-196, is then one pass), else their own pass
  normalize(pending);
  if (!pending.identity()) {
    Pass* last = plan.passes.empty() ? nullptr : &plan.passes.back();
    const bool epi_ok = fuse && last &&
                        (last->kind == PassKind::Separable || last->kind == PassKind::Direct) &&
                        !last->has_epi && !last->epi_expand && !pending.gray && !pending.has_pre &&
                        (!pending.expand || last->cmid == 1);
    if (epi_ok) {
      if (pending.has_post) {
        last->has_epi = true;
        last->epi = pending.post;
      }
      if (pending.expand) {
        last->epi_expand = true;
        last->cout = 3;
      }
      last->desc += " epilogue[" + prog_desc(pending) + "]";
      pending = PointwiseProgram{};
    } else {
      flush_pointwise();
    }
  }
  if (plan.passes.empty()) {  // identity chain: keep one copy pass so outputs are fresh
    Pass p;
    p.kind = PassKind::Pointwise;
    p.cin = p.cout = p.cmid = c;
    p.desc = "pointwise[copy]";
    plan.passes.push_back(p);
  }
  plan.cout = c;

  // halo/margin contracts: each pass's output margins serve the next stencil consumer
  int next_r = 0;
  Border next_b = Border::Reflect101;
  for (int i = (int)plan.passes.size() - 1; i >= 0; --i) {
    Pass& p = plan.passes[i];
    p.out_margin_px = next_r;
    p.out_margin_border = next_b;
    if (p.kind != PassKind::Pointwise) {
      next_r = p.R;
      next_b = p.border == Border::Skip ? Border::Reflect101 : p.border;
    }
  }
  plan.in_margin_px = next_r;
  plan.in_margin_border = next_b;
  // a chain that maps C -> C can be iterated (ping-pong): the last pass then
  // feeds the first one, so it must maintain the first pass's input margins.
  // A pointwise pass maps its input margins byte by byte, so the contract
  // walks back through the trailing pointwise passes to the last stencil/conv
  // pass, which recomputes its output margins from its own pixels.
  if (plan.cout == plan.cin && plan.in_margin_px > 0) {
    for (int i = (int)plan.passes.size() - 1; i >= 0; --i) {
      Pass& p = plan.passes[i];
      if (p.out_margin_px < plan.in_margin_px) {
        p.out_margin_px = plan.in_margin_px;
        p.out_margin_border = plan.in_margin_border;
      }
      if (p.kind != PassKind::Pointwise) break;
    }
  }
  plan.max_radius = 0;
  plan.max_channels = cin;
  for (const Pass& p : plan.passes) {
    plan.max_radius = std::max(plan.max_radius, p.R);
    plan.max_channels = std::max(plan.max_channels, std::max(p.cin, p.cout));
  }
  // a pointwise pass cannot move a margin across a channel change: 3->1 keeps
  // margins valid (per pixel), and every C stores >= kMaxRadius... check it.
  for (const Pass& p : plan.passes)
    STRIPE_CHECK(p.out_margin_px <= margin_pixels(p.cout), "margin contract too wide");
  for (Pass& p : plan.passes)
    if (p.kind != PassKind::Pointwise && p.pro.has_post && p.pro.gray && p.pro.gmode == GrayMode::Ref) {
      p.post_aff = lut_affine(p.pro.post, &p.post_a, &p.post_b, &p.post_k);
      if (p.post_aff)
        p.desc += " post=clamp((" + std::to_string(p.post_a) + "v" + (p.post_b < 0 ? "" : "+") +
                  std::to_string(p.post_b) + ")>>" + std::to_string(p.post_k) + ")";
    }
  return plan;
}

bool lut_affine(const std::array<uint8_t, 256>& lut, int* a_out, int* b_out, int* k_out) {
  for (int k = 0; k <= 8; ++k) {
    const int64_t q = int64_t(1) << k;
    for (int a = -255; a <= 255; ++a) {
      // b range from the unclamped entries: L q <= a v + b < (L + 1) q
      int64_t lo = INT32_MIN, hi = INT32_MAX;
      for (int v = 0; v < 256 && lo <= hi; ++v) {
        const int L = lut[v];
        if (L == 0 || L == 255) continue;
        lo = std::max(lo, L * q - (int64_t)a * v);
        hi = std::min(hi, (L + 1) * q - 1 - (int64_t)a * v);
      }
      if (lo > hi) continue;
      // a constant-free table (all entries clamped) leaves b open: try the
      // range's ends and a few values in between
      const int64_t cands[3] = {lo == INT32_MIN ? -32767 : lo, hi == INT32_MAX ? 32767 : hi,
                                lo == INT32_MIN || hi == INT32_MAX ? 0 : (lo + hi) / 2};
      for (int64_t b : cands) {
        if (std::llabs(b) + 255LL * std::abs(a) >= 32768) continue;
        bool ok = true;
        for (int v = 0; v < 256 && ok; ++v) {
          int64_t t = ((int64_t)a * v + b);
          t = t >= 0 ? t >> k : -((-t + q - 1) >> k);  // arithmetic shift = floor
          t = std::min<int64_t>(255, std::max<int64_t>(0, t));
          ok = t == lut[v];
        }
        if (ok) {
          *a_out = a;
          *b_out = (int)b;
          *k_out = k;
          return true;
        }
      }
    }
  }
  return false;
}

}  // namespace stripe
