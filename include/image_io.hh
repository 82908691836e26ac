// image_io.hh — the reference's Image container, declaration-compatible with
// ahmedhassayoune/sift-project src/image_io.hh:22-52 so that code compiled
// against either header links against the same objects.
//
// Layout: interleaved HWC doubles, data[(y*width + x)*channels + c]
// (reference image_io.cpp:81-92). Pixel values are 0..255 as decoded by
// stbi_load(..., 0) with channels capped at 3 (image_io.cpp:22-33).
//
// The drop-in replaces the reference's src/sift.cpp only; the Image member
// functions (load/save via stb, pixel accessors, drawing) stay the
// reference's own image_io.cpp / image.cpp. This header therefore declares
// them but does not pull in stb.
#pragma once

#include <iostream>
#include <string>
#include <vector>

enum Channel { R = 0, G = 1, B = 2, GRAY = 0 };

enum ImageFormat { PNG, BMP, TGA, JPG };

enum Color {
    BLACK = 0,
    WHITE = 0xFFFFFF,
    RED = 0xFF0000,
    GREEN = 0x00FF00,
    BLUE = 0x0000FF,
    YELLOW = 0xFFFF00,
    CYAN = 0x00FFFF,
    MAGENTA = 0xFF00FF
};

struct Image {
    int width;
    int height;
    int channels;
    std::vector<double> data;

    // construction / loading (image_io.cpp:9-68)
    Image();
    Image(int w, int h, int c);
    Image(const char* filename);
    Image(std::string filename);
    Image(const Image& other);
    Image(Image&& other);
    Image& operator=(const Image& other);
    size_t size() const;

    // pixel access and saving (image_io.cpp:72-154)
    double get_pixel(int x, int y, Channel c) const;
    void set_pixel(int x, int y, Channel c, double value);
    bool save(const char* filename, const ImageFormat format = PNG) const;
    bool save(const std::string filename, const ImageFormat format = PNG) const;
    double operator()(int x, int y, Channel c) const;
    double operator()(int x, int y) const;

    // drawing (image.cpp:245-328)
    void draw_point(int x, int y, int size, int color = RED);
    void draw_circle(int x, int y, int radius, int color = RED, int thickness = 1);
    void draw_line(int x1, int y1, int x2, int y2, int color = RED, int thickness = 1);
};
