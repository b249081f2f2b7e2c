// Cartesian process topology: the MPI_Dims_create / Cart_coords / Cart_shift
// semantics that the reference obtains from libmpi
// (src/init_global_grid.jl:84-93), re-implemented as pure host math so the
// topology needs no MPI and is testable without any communicator.
//
// Rank <-> coords mapping: row-major, last dimension fastest (MPI standard;
// SURVEY.md §2.4 invariant 12). `reorder` is accepted and ignored.
#pragma once

#include <array>
#include <cstdint>
#include <vector>

#include "igg/common.hpp"

namespace igg {

using Int3 = std::array<int64_t, NDIMS>;

// Fill the zero entries of `dims` so that prod(dims) == nprocs, as balanced as
// possible, free entries in non-increasing order (MPI_Dims_create contract).
// Throws igg::Error if nprocs is not divisible by the product of fixed entries.
Int3 dims_create(int64_t nprocs, Int3 dims);

// Row-major Cartesian coordinates of `rank` in a grid of `dims`.
Int3 cart_coords(int64_t rank, const Int3& dims);

// Inverse of cart_coords (coords must be in range).
int64_t cart_rank(const Int3& coords, const Int3& dims);

// (source, dest) neighbours of `rank` along `dim` for displacement `disp`
// (MPI_Cart_shift). Non-periodic out-of-range neighbours are PROC_NULL.
std::array<int64_t, 2> cart_shift(int64_t rank, int dim, int64_t disp,
                                  const Int3& dims, const Int3& periods);

// Implicit global grid size: dims*(nxyz-overlaps) + overlaps*(periods==0)
// (init_global_grid.jl:93).
Int3 global_size(const Int3& nxyz, const Int3& dims, const Int3& overlaps,
                 const Int3& periods);

// Global coordinate of local index `i` (0-based) of an array whose size along
// `dim` is `size_a` (tools.jl:98-107; staggered offset, rank shift, periodic
// wrap). `n`, `ol`, `coord`, `n_g`, `periodic` are the grid values of `dim`.
double coord_g(int64_t i, double d, int64_t size_a, int64_t n, int64_t ol,
               int64_t coord, int64_t n_g, bool periodic);

}  // namespace igg
