// oracle/ref_harness.cpp — TEST INFRASTRUCTURE ONLY, builds in this
// container only (needs /root/reference). Output binaries go to oracle/_ref/.
//
// A driver TU that textually includes the reference's src/sift.cpp (path in
// REF_SIFT_CPP, see oracle/Makefile; nothing is copied into this repo) so it
// can reach the anonymous-namespace stage functions (sift.cpp:7-697) and run
// them in the order of detect_keypoints_and_descriptors (sift.cpp:717-771),
// dumping every intermediate. It skips only the keypoints.png draw/save
// (sift.cpp:765-768) and silences the progress prints.
//
// The "copy-fixed" build (ref_harness_cf) streams sift.cpp through sed to
// turn the four per-item deep copies (sift.cpp:311,346,466,616) into const
// references (outputs verified byte-identical to the as-is build by
// tests/golden/make_goldens.py) and to insert SIFT_DESC_HOOK in
// convert_hist_to_desc (sift.cpp:600) to capture the normalised descriptor
// floats h*norm_inv that the reference never exposes.
//
// usage: ref_harness <input> <out_prefix> [intervals=3] [double=1]
//                    [max_octaves=0] [dump_pyramid=0]
//                    [window_size=3] [init_sigma=1.6] [contrast_threshold=0.04]
//                    [eigen_ratio=10] [num_bins=36] [peak_ratio=0.8]
//                    [ori_sigma_factor=1.5] [desc_scale_factor=3]
//        ref_harness --match <kps1.bin> <kps2.bin> <ratio> <out.bin>
//   (the trailing arguments are the remaining parameters of
//   detect_keypoints_and_descriptors, reference sift.hh:65-71, parsed with
//   strtod so every double round-trips exactly from its repr)
//   <input> is an image file (stb decode, image_io.cpp:20-35) or a raw file
//   "SIFTRAW1" + int32 w,h,c + w*h*c little-endian doubles.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

static std::vector<float> g_desc_hook;
#define SIFT_DESC_HOOK(v) g_desc_hook.push_back((float)(v))

#include REF_SIFT_CPP

#include <chrono>

namespace {

bool read_raw(const char* path, Image& img) {
    std::ifstream f(path, std::ios::binary);
    char magic[8];
    if (!f.read(magic, 8) || std::memcmp(magic, "SIFTRAW1", 8) != 0) return false;
    int32_t dims[3];
    f.read(reinterpret_cast<char*>(dims), sizeof dims);
    img = Image(dims[0], dims[1], dims[2]);
    f.read(reinterpret_cast<char*>(img.data.data()), sizeof(double) * img.data.size());
    return (bool)f;
}

void write_raw(const std::string& path, const Image& img) {
    std::ofstream f(path, std::ios::binary);
    f.write("SIFTRAW1", 8);
    int32_t dims[3] = {img.width, img.height, img.channels};
    f.write(reinterpret_cast<const char*>(dims), sizeof dims);
    f.write(reinterpret_cast<const char*>(img.data.data()), sizeof(double) * img.data.size());
}

template <class T>
void write_vec(const std::string& path, const std::vector<T>& v) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(v.data()), sizeof(T) * v.size());
}

struct ExtRec {
    int32_t x, y, z, o;
};

}  // namespace

// --match <kps1.bin> <kps2.bin> <ratio> <out.bin>: the reference
// match_keypoints (sift.cpp:783-815) on two raw Keypoint arrays; writes one
// (int32 i1, int32 i2, double distance) triple per match, the indices
// recovered by byte comparison of the copies KeypointMatch holds.
int match_mode(char** argv) {
    auto load = [](const char* path) {
        std::ifstream f(path, std::ios::binary | std::ios::ate);
        const size_t bytes = (size_t)f.tellg();
        std::vector<Keypoint> v(bytes / sizeof(Keypoint));
        f.seekg(0);
        f.read(reinterpret_cast<char*>(v.data()), v.size() * sizeof(Keypoint));
        return v;
    };
    const std::vector<Keypoint> a = load(argv[2]), b = load(argv[3]);
    const double ratio = std::atof(argv[4]);
    std::streambuf* saved = std::cout.rdbuf(nullptr);
    const std::vector<KeypointMatch> m = match_keypoints(a, b, ratio);
    std::cout.rdbuf(saved);
    std::ofstream f(argv[5], std::ios::binary);
    size_t i1 = 0;
    for (const KeypointMatch& k : m) {
        while (i1 < a.size() && std::memcmp(&a[i1], &k.kp1, sizeof(Keypoint)) != 0) ++i1;
        size_t i2 = 0;
        while (i2 < b.size() && std::memcmp(&b[i2], &k.kp2, sizeof(Keypoint)) != 0) ++i2;
        if (i1 == a.size() || i2 == b.size()) return 3;
        const int32_t idx[2] = {(int32_t)i1, (int32_t)i2};
        f.write(reinterpret_cast<const char*>(idx), sizeof idx);
        f.write(reinterpret_cast<const char*>(&k.distance), sizeof(double));
        ++i1;
    }
    std::printf("match: %zu x %zu -> %zu\n", a.size(), b.size(), m.size());
    return 0;
}

int main(int argc, char** argv) {
    if (argc == 6 && std::strcmp(argv[1], "--match") == 0) return match_mode(argv);
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <input> <out_prefix> [intervals] [double] [max_octaves] [dump_pyr]\n", argv[0]);
        return 2;
    }
    const std::string out = argv[2];
    const int intervals = argc > 3 ? std::atoi(argv[3]) : 3;
    const bool dbl = argc > 4 ? std::atoi(argv[4]) != 0 : true;
    const int max_oct = argc > 5 ? std::atoi(argv[5]) : 0;
    const bool dump_pyr = argc > 6 ? std::atoi(argv[6]) != 0 : false;
    // reference defaults, sift.hh:65-71, unless given
    auto dbl_arg = [&](int i, double d) { return argc > i ? std::strtod(argv[i], nullptr) : d; };
    const int window_size = argc > 7 ? std::atoi(argv[7]) : 3;
    const double init_sigma = dbl_arg(8, 1.6), ct = dbl_arg(9, 0.04), er = dbl_arg(10, 10.0),
                 num_bins = dbl_arg(11, 36), peak_ratio = dbl_arg(12, 0.8),
                 ori_sf = dbl_arg(13, 1.5), desc_sf = dbl_arg(14, 3.0);

    Image img;
    if (!read_raw(argv[1], img)) {
        img = Image(argv[1]);
        write_raw(out + ".input.raw", img);
    }
    std::streambuf* saved = std::cout.rdbuf(nullptr);  // silence progress prints

    using clk = std::chrono::steady_clock;
    auto t0 = clk::now();
    Image initial = compute_initial_image(img, dbl, init_sigma);
    int octaves = compute_octaves_count(initial.width, initial.height);
    if (max_oct > 0 && octaves > max_oct) octaves = max_oct;
    std::vector<double> kernels = compute_gaussian_kernels(init_sigma, intervals);
    auto t1 = clk::now();
    auto gauss = compute_gaussian_images(initial, octaves, kernels);
    auto t2 = clk::now();
    auto dog = compute_dog_images(gauss, octaves, intervals);
    auto t3 = clk::now();
    auto extrema = detect_extrema(dog, kernels, intervals, window_size, ct);
    auto t4 = clk::now();
    auto kps = compute_keypoints(dog, extrema, kernels, init_sigma, window_size,
                                 intervals, ct, er);
    auto t5 = clk::now();
    std::vector<Keypoint> refined = kps;
    kps = compute_orientations(kps, kernels, gauss, num_bins, peak_ratio, ori_sf, dbl);
    auto t6 = clk::now();
    std::vector<Keypoint> oriented = kps;
    clean_keypoints(kps);
    auto t7 = clk::now();
    compute_descriptors(kps, gauss, desc_sf, dbl);
    auto t8 = clk::now();
    std::cout.rdbuf(saved);

    auto s = [](clk::time_point a, clk::time_point b) {
        return std::chrono::duration<double>(b - a).count();
    };
    std::vector<ExtRec> ext;
    for (const auto& e : extrema)
        ext.push_back({(int32_t)std::get<0>(e), (int32_t)std::get<1>(e),
                       (int32_t)std::get<2>(e), (int32_t)std::get<3>(e)});
    write_vec(out + ".ext.bin", ext);
    write_vec(out + ".refined.bin", refined);
    write_vec(out + ".oriented.bin", oriented);
    write_vec(out + ".final.bin", kps);
    if (!g_desc_hook.empty()) write_vec(out + ".df32.bin", g_desc_hook);
    if (dump_pyr) {
        std::ofstream f(out + ".pyr.bin", std::ios::binary);
        for (const auto& oct : gauss)
            for (const auto& lvl : oct)
                f.write(reinterpret_cast<const char*>(lvl.data.data()),
                        sizeof(double) * lvl.data.size());
    }
    std::ofstream m(out + ".meta.txt");
    m << "width " << img.width << "\nheight " << img.height << "\nchannels "
      << img.channels << "\nintervals " << intervals << "\ndouble " << dbl
      << "\nmax_octaves " << max_oct << "\noctaves " << octaves << "\nlevels "
      << kernels.size() << "\n";
    for (int o = 0; o < octaves; ++o)
        m << "octave_dims " << o << " " << gauss[o][0].width << " " << gauss[o][0].height << "\n";
    m << "extrema " << extrema.size() << "\nrefined " << refined.size()
      << "\noriented " << oriented.size() << "\nfinal " << kps.size() << "\n";
    m << "sizeof_keypoint " << sizeof(Keypoint) << "\n";
    m.precision(6);
    m << "time_init " << s(t0, t1) << "\ntime_pyramid " << s(t1, t2)
      << "\ntime_dog " << s(t2, t3) << "\ntime_extrema " << s(t3, t4)
      << "\ntime_refine " << s(t4, t5) << "\ntime_orient " << s(t5, t6)
      << "\ntime_clean " << s(t6, t7) << "\ntime_desc " << s(t7, t8)
      << "\ntime_total " << s(t0, t8) << "\n";
    std::printf("%s: octaves=%d extrema=%zu refined=%zu oriented=%zu final=%zu total=%.3fs\n",
                out.c_str(), octaves, extrema.size(), refined.size(), oriented.size(),
                kps.size(), s(t0, t8));
    return 0;
}
