// Cartesian topology math (see include/igg/topology.hpp).
// Reference behaviour: init_global_grid.jl:84-93 (MPI.Dims_create!, Cart_create,
// Cart_coords, Cart_shift and nxyz_g = dims.*(nxyz.-overlaps) .+ overlaps.*(periods.==0)).
// No MPI here: balanced dims, row-major coords and shifts are computed directly.
#include "igg/topology.hpp"

#include <algorithm>
#include <functional>

namespace igg {

namespace {
std::vector<int64_t> prime_factors(int64_t n) {
  std::vector<int64_t> f;
  for (int64_t p = 2; p * p <= n; ++p)
    while (n % p == 0) { f.push_back(p); n /= p; }
  if (n > 1) f.push_back(n);
  return f;
}
}  // namespace

Int3 dims_create(int64_t nprocs, Int3 dims) {
  if (nprocs < 1) fail("dims_create: nprocs must be >= 1 (got ", nprocs, ").");
  int64_t fixed = 1;
  std::vector<int> free_idx;
  for (int d = 0; d < NDIMS; ++d) {
    if (dims[d] < 0) fail("dims_create: negative dims entry (", dims[d], ").");
    if (dims[d] == 0) free_idx.push_back(d); else fixed *= dims[d];
  }
  if (nprocs % fixed != 0)
    fail("dims_create: nprocs (", nprocs, ") is not divisible by the product of the fixed dims (",
         fixed, ").");
  int64_t rest = nprocs / fixed;
  if (free_idx.empty()) {
    if (rest != 1)
      fail("dims_create: the fixed dims product (", fixed, ") does not match nprocs (", nprocs, ").");
    return dims;
  }
  // Greedy balanced factorisation: largest prime first onto the currently
  // smallest free dimension; then sort free entries non-increasingly.
  std::vector<int64_t> fac = prime_factors(rest);
  std::sort(fac.begin(), fac.end(), std::greater<int64_t>());
  std::vector<int64_t> vals(free_idx.size(), 1);
  for (int64_t p : fac) {
    auto it = std::min_element(vals.begin(), vals.end());
    *it *= p;
  }
  std::sort(vals.begin(), vals.end(), std::greater<int64_t>());
  for (size_t k = 0; k < free_idx.size(); ++k) dims[free_idx[k]] = vals[k];
  return dims;
}

Int3 cart_coords(int64_t rank, const Int3& dims) {
  Int3 c{};
  int64_t r = rank;
  for (int d = NDIMS - 1; d >= 0; --d) {
    c[d] = r % dims[d];
    r /= dims[d];
  }
  return c;
}

int64_t cart_rank(const Int3& coords, const Int3& dims) {
  int64_t r = 0;
  for (int d = 0; d < NDIMS; ++d) r = r * dims[d] + coords[d];
  return r;
}

std::array<int64_t, 2> cart_shift(int64_t rank, int dim, int64_t disp,
                                  const Int3& dims, const Int3& periods) {
  if (dim < 0 || dim >= NDIMS) fail("cart_shift: invalid dim ", dim);
  Int3 c = cart_coords(rank, dims);
  std::array<int64_t, 2> out{};
  for (int s = 0; s < 2; ++s) {
    int64_t cc = c[dim] + (s == 0 ? -disp : disp);
    if (cc < 0 || cc >= dims[dim]) {
      if (!periods[dim]) { out[s] = PROC_NULL; continue; }
      cc = ((cc % dims[dim]) + dims[dim]) % dims[dim];
    }
    Int3 n = c;
    n[dim] = cc;
    out[s] = cart_rank(n, dims);
  }
  return out;
}

Int3 global_size(const Int3& nxyz, const Int3& dims, const Int3& overlaps,
                 const Int3& periods) {
  Int3 g{};
  for (int d = 0; d < NDIMS; ++d)
    g[d] = dims[d] * (nxyz[d] - overlaps[d]) + overlaps[d] * (periods[d] == 0 ? 1 : 0);
  return g;
}

double coord_g(int64_t i, double d, int64_t size_a, int64_t n, int64_t ol,
               int64_t coord, int64_t n_g, bool periodic) {
  const double x0 = 0.5 * static_cast<double>(n - size_a) * d;
  double x = static_cast<double>(coord * (n - ol) + i) * d + x0;
  if (periodic) {
    x -= d;
    if (x > static_cast<double>(n_g - 1) * d) x -= static_cast<double>(n_g) * d;
    if (x < 0) x += static_cast<double>(n_g) * d;
  }
  return x;
}

}  // namespace igg
