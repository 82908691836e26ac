// image.hh — image operations of the reference (src/image.hh:5-13),
// declared for source compatibility. They are implemented by the
// reference's own image.cpp, which the drop-in keeps; on MI355X the ones on
// the SIFT hot path (grayscale, bilinear x2, nearest /2, separable Gaussian,
// subtract) run fused inside the HIP kernels instead (sift_kernels.hip).
#pragma once

#include "image_io.hh"

Image convert_to_grayscale(const Image& img);
Image subtract(const Image& img1, const Image& img2);
Image resize_inter_nearest(const Image& img);
Image resize_inter_bilinear(const Image& img, int fx, int fy);
Image apply_convolution(const Image& img, const std::vector<double>& kernel);
Image apply_double_convolution_1d(const Image& img, const std::vector<double>& kernel);
Image apply_gaussian_blur(const Image& img, double sigma);
Image apply_gaussian_blur_fast(const Image& img, double sigma);
