// Winograd F(m x m, 3 x 3) transform matrices (Lavin & Gray): B^T (input,
// (m+2) x (m+2)) and A^T (output, m x (m+2)), shared by the transform kernels
// of conv.hip and wino_fused.hip.
#pragma once

namespace mdx {

template <int M>
struct WinoT;
template <>
struct WinoT<2> {
    static constexpr int A = 4;
    __device__ static constexpr float BT(int i, int j) {
        constexpr float t[4][4] = {{1, 0, -1, 0}, {0, 1, 1, 0}, {0, -1, 1, 0}, {0, 1, 0, -1}};
        return t[i][j];
    }
    __device__ static constexpr float AT(int i, int j) {
        constexpr float t[2][4] = {{1, 1, 1, 0}, {0, 1, -1, -1}};
        return t[i][j];
    }
};
template <>
struct WinoT<4> {
    static constexpr int A = 6;
    __device__ static constexpr float BT(int i, int j) {
        constexpr float t[6][6] = {{4, 0, -5, 0, 1, 0},  {0, -4, -4, 1, 1, 0}, {0, 4, -4, -1, 1, 0},
                                   {0, -2, -1, 2, 1, 0}, {0, 2, -1, -2, 1, 0}, {0, 4, 0, -5, 0, 1}};
        return t[i][j];
    }
    __device__ static constexpr float AT(int i, int j) {
        constexpr float t[4][6] = {{1, 1, 1, 1, 1, 0}, {0, 1, -1, 2, -2, 0}, {0, 1, 1, 4, 4, 0}, {0, 1, -1, 8, -8, 1}};
        return t[i][j];
    }
};
template <>
struct WinoT<6> {
    static constexpr int A = 8;
    __device__ static constexpr float BT(int i, int j) {
        constexpr float t[8][8] = {{1, 0, -5.25f, 0, 5.25f, 0, -1, 0},       {0, 1, 1, -4.25f, -4.25f, 1, 1, 0},
                                   {0, -1, 1, 4.25f, -4.25f, -1, 1, 0},      {0, 0.5f, 0.25f, -2.5f, -1.25f, 2, 1, 0},
                                   {0, -0.5f, 0.25f, 2.5f, -1.25f, -2, 1, 0}, {0, 2, 4, -2.5f, -5, 0.5f, 1, 0},
                                   {0, -2, 4, 2.5f, -5, -0.5f, 1, 0},        {0, -1, 0, 5.25f, 0, -5.25f, 0, 1}};
        return t[i][j];
    }
    __device__ static constexpr float AT(int i, int j) {
        constexpr float t[6][8] = {{1, 1, 1, 1, 1, 1, 1, 0},
                                   {0, 1, -1, 2, -2, 0.5f, -0.5f, 0},
                                   {0, 1, 1, 4, 4, 0.25f, 0.25f, 0},
                                   {0, 1, -1, 8, -8, 0.125f, -0.125f, 0},
                                   {0, 1, 1, 16, 16, 0.0625f, 0.0625f, 0},
                                   {0, 1, -1, 32, -32, 0.03125f, -0.03125f, 1}};
        return t[i][j];
    }
};

}  // namespace mdx
