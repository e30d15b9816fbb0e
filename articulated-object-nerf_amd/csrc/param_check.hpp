// Shape checks of the MLP parameter tables (include/aonerf.h aon_mlp_params /
// aon_mlp_art_params, ABI 9), run by every pack before it launches anything: a mis-ordered or
// mis-shaped parameter list (e.g. nn.Module.parameters() in registration order, which is not the
// kernels' layer order) returns < 0 with the offending layer named, instead of a pack kernel
// reading past the end of a tensor (the round-4 illegal-address fault).
#pragma once

#include <string>

#include "aon_common.hpp"

namespace aon {
namespace mlp {

// expected [out][in] of the vanilla NeRFMLP (reference model.py:39-93, default geometry), in
// the field order of aon_mlp_params
constexpr int kVanillaShape[12][2] = {{256, 63},  {256, 256}, {256, 256}, {256, 256},
                                      {256, 256}, {256, 319}, {256, 256}, {256, 256},
                                      {1, 256},   {256, 256}, {128, 283}, {3, 128}};
constexpr const char* kVanillaName[12] = {
    "pts_linears.0", "pts_linears.1", "pts_linears.2", "pts_linears.3",
    "pts_linears.4", "pts_linears.5", "pts_linears.6", "pts_linears.7",
    "density_layer", "bottleneck_layer", "views_linear.0", "rgb_layer"};

// the articulated NeRFMLP (model_autodecoder.py:60-166): [out][per-sample in]; `latent` marks
// the four layers whose rows continue with latent columns (folded into the bias by the caller),
// whose width must be at least the per-sample columns
struct ArtShape {
  int out, in;
  bool latent;
  const char* name;
};
constexpr ArtShape kArtShape[20] = {
    {128, 3, true, "deformations_linear.0"}, {128, 128, false, "deformations_linear.1"},
    {128, 128, false, "deformations_linear.2"}, {128, 128, false, "deformations_linear.3"},
    {3, 128, false, "deformation_layer"},    {256, 63, true, "pts_linears.0"},
    {256, 256, false, "pts_linears.1"},      {256, 256, false, "pts_linears.2"},
    {256, 256, false, "pts_linears.3"},      {256, 256, false, "pts_linears.4"},
    {256, 319, true, "pts_linears.5"},       {256, 256, false, "pts_linears.6"},
    {256, 256, false, "pts_linears.7"},      {1, 256, false, "density_layer"},
    {256, 256, false, "bottleneck_layer"},   {128, 283, true, "views_linear.0"},
    {128, 128, false, "views_linear.1"},     {128, 128, false, "views_linear.2"},
    {128, 128, false, "views_linear.3"},     {3, 128, false, "rgb_layer"}};

inline int shape_error(const char* fn, const char* layer, int64_t rows, int64_t cols, int64_t blen,
                       int out, int in, bool at_least) {
  set_error(std::string(fn) + ": " + layer + ": weight " + std::to_string(rows) + " x " +
            std::to_string(cols) + ", bias " + std::to_string(blen) + "; expected weight " +
            std::to_string(out) + " x " + (at_least ? ">= " : "") + std::to_string(in) +
            ", bias " + std::to_string(out) +
            " (parameters in the kernels' layer order, include/aonerf.h)");
  return -1;
}

inline int check_mlp_params(const aon_mlp_params* p, const char* fn) {
  for (int i = 0; i < 12; ++i) {
    const int out = kVanillaShape[i][0], in = kVanillaShape[i][1];
    if (p->w_rows[i] != out || p->w_cols[i] != in || p->b_len[i] != out)
      return shape_error(fn, kVanillaName[i], p->w_rows[i], p->w_cols[i], p->b_len[i], out, in,
                         false);
  }
  return 0;
}

inline int check_mlp_art_params(const aon_mlp_art_params* p, const char* fn) {
  for (int i = 0; i < 20; ++i) {
    const ArtShape& s = kArtShape[i];
    const bool cols_ok = s.latent ? p->w_cols[i] >= s.in : p->w_cols[i] == s.in;
    if (p->w_rows[i] != s.out || !cols_ok || p->b_len[i] != s.out || p->w_cols[i] > (1 << 20))
      return shape_error(fn, s.name, p->w_rows[i], p->w_cols[i], p->b_len[i], s.out, s.in,
                         s.latent);
  }
  return 0;
}

// row strides of the latent-carrying articulated weights (their full widths)
enum { kArtDef0 = 0, kArtPts0 = 5, kArtPts5 = 10, kArtView0 = 15 };

}  // namespace mlp
}  // namespace aon
