/*
 * TEST INFRASTRUCTURE ONLY -- replays /root/reference/test/test_gicp_alignment.cpp:50-131 through
 * the drop-in adapter class itself (adapter/GICPAlignment.cpp over libmgicp.so), plus the two
 * Filter members of adapter/Filter_mi355x.cpp.  gtest is absent from this image, so EXPECT /
 * ASSERT are restated as counted checks; every transform is printed for the Python side
 * (tests/test_adapter_build.py) to compare with the oracle.
 *
 * usage: replay SOURCE.bin TARGET.bin      (n x 3 float32 each: the fixture of :32-47)
 *        replay --no-device                (no GPU: the adapter must fail soft, as PCL errors do)
 * output lines:  "<case> T <16 floats, column-major> exists <0|1>"  and  "<check> ok|FAIL"
 */
#include <GICPAlignment.h>
#include <Filter.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>

typedef pcl::PointCloud<pcl::PointXYZRGB> PointCloudRGB;

static int g_fail = 0;

static void check(bool ok, const char* what)
{
    std::printf("%s %s\n", what, ok ? "ok" : "FAIL");
    if (!ok)
        ++g_fail;
}

static void print_tf(const char* name, const Eigen::Matrix4f& T, bool exists)
{
    std::printf("%s T", name);
    for (int i = 0; i < 16; ++i)
        std::printf(" %.9g", T.data()[i]);
    std::printf(" exists %d\n", exists ? 1 : 0);
}

static PointCloudRGB::Ptr load(const char* path)
{
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f)
    {
        std::fprintf(stderr, "cannot open %s\n", path);
        std::exit(2);
    }
    const std::streamsize bytes = f.tellg();
    f.seekg(0);
    std::vector<float> xyz(static_cast<size_t>(bytes) / sizeof(float));
    f.read(reinterpret_cast<char*>(xyz.data()), bytes);
    PointCloudRGB::Ptr c(new PointCloudRGB);
    for (size_t i = 0; i + 2 < xyz.size(); i += 3)
    {
        pcl::PointXYZRGB p;
        p.x = xyz[i];
        p.y = xyz[i + 1];
        p.z = xyz[i + 2];
        p.r = p.g = p.b = 255;
        c->push_back(p);
    }
    return c;
}

static bool same_xyz(const PointCloudRGB& a, const PointCloudRGB& b)
{
    if (a.points.size() != b.points.size())
        return false;
    for (size_t i = 0; i < a.points.size(); ++i)
        if (a.points[i].x != b.points[i].x || a.points[i].y != b.points[i].y || a.points[i].z != b.points[i].z)
            return false;
    return true;
}

int main(int argc, char** argv)
{
    static_assert(sizeof(pcl::PointXYZRGB) == 32, "layout");
    static_assert(offsetof(pcl::PointXYZRGB, rgba) == 16, "layout");
    if (argc == 2 && std::string(argv[1]) == "--no-device")
    {
        // mgicp_create fails without a HIP device: the class must construct, log, and report
        // "no transform" exactly like a PCL solver failure (transform_exists_ stays false)
        PointCloudRGB::Ptr a(new PointCloudRGB), b(new PointCloudRGB);
        for (int i = 0; i < 64; ++i)
        {
            pcl::PointXYZRGB p;
            p.x = 0.01f * i;
            p.y = 0.02f * (i % 7);
            p.z = 0.03f * (i % 5);
            a->push_back(p);
            b->push_back(p);
        }
        GICPAlignment g(a, b, false);
        check(g.getFineTransform() == Eigen::Matrix4f::Identity(), "nodev_ctor_identity");
        g.run();
        check(!g.transform_exists_, "nodev_no_transform");
        return g_fail ? 1 : 0;
    }
    if (argc != 3)
    {
        std::fprintf(stderr, "usage: %s SOURCE.bin TARGET.bin | --no-device\n", argv[0]);
        return 2;
    }
    PointCloudRGB::Ptr sourceRGB0 = load(argv[1]);
    PointCloudRGB::Ptr targetRGB0 = load(argv[2]);

    {  // testApplyTF (:50-75)
        PointCloudRGB::Ptr sourceRGB(new PointCloudRGB(*sourceRGB0)), targetRGB(new PointCloudRGB(*targetRGB0));
        GICPAlignment gicp_alignment(targetRGB, sourceRGB, false);
        check(gicp_alignment.getFineTransform() == Eigen::Matrix4f::Identity(), "testApplyTF_ctor_identity");
        ros::Time::init();
        gicp_alignment.run();
        const PointCloudRGB before = *sourceRGB;
        gicp_alignment.applyTFtoCloud(sourceRGB);
        // applyTFtoCloud writes aligned_cloud_, not its argument (src/GICPAlignment.cpp:144-147)
        check(same_xyz(before, *sourceRGB), "testApplyTF_argument_untouched");
        PointCloudRGB::Ptr aligned(new PointCloudRGB);
        gicp_alignment.getAlignedCloud(aligned);
        check(aligned->points.size() == sourceRGB->points.size(), "testApplyTF_aligned_size");
        print_tf("testApplyTF", gicp_alignment.getFineTransform(), gicp_alignment.transform_exists_);
        // aligned_cloud_ = fine_tf * source, first point
        const Eigen::Matrix4f T = gicp_alignment.getFineTransform();
        const pcl::PointXYZRGB& s = sourceRGB->points[0];
        float x = T(0, 0) * s.x;
        x = x + T(0, 1) * s.y;
        x = x + T(0, 2) * s.z;
        x = x + T(0, 3);
        check(aligned->points[0].x == x, "testApplyTF_aligned_first_point");
        check(gicp_alignment.transform_exists_, "testApplyTF_exists");
    }
    {  // testRun (:77-104): the int setters truncate 5e-2 -> 0
        PointCloudRGB::Ptr sourceRGB(new PointCloudRGB(*sourceRGB0)), targetRGB(new PointCloudRGB(*targetRGB0));
        GICPAlignment gicp_alignment(targetRGB, sourceRGB, false);
        check(gicp_alignment.getFineTransform() == Eigen::Matrix4f::Identity(), "testRun_ctor_identity");
        gicp_alignment.setMaxIterations(100);
        gicp_alignment.setMaxCorrespondenceDistance(5);
        gicp_alignment.setRANSACOutlierTh(5e-2);
        gicp_alignment.setTfEpsilon(5e-4);
        ros::Time::init();
        gicp_alignment.run();
        PointCloudRGB::Ptr aligned_cloud(new PointCloudRGB);
        gicp_alignment.getAlignedCloud(aligned_cloud);
        check(gicp_alignment.transform_exists_, "testRun_exists");
        check(aligned_cloud->points.size() == sourceRGB->points.size(), "testRun_aligned_size");
        sensor_msgs::PointCloud2 msg;
        gicp_alignment.getAlignedCloudROSMsg(msg);
        check(msg.width == sourceRGB->points.size() && msg.point_step == 32, "testRun_ros_msg");
        print_tf("testRun", gicp_alignment.getFineTransform(), gicp_alignment.transform_exists_);
    }
    {  // testRunWithCov (:106-131): run() with covariances, then iterate(): fine_tf = T * T
        PointCloudRGB::Ptr sourceRGB(new PointCloudRGB(*sourceRGB0)), targetRGB(new PointCloudRGB(*targetRGB0));
        GICPAlignment gicp_alignment(targetRGB, sourceRGB, true);
        check(gicp_alignment.getFineTransform() == Eigen::Matrix4f::Identity(), "testRunWithCov_ctor_identity");
        ros::Time::init();
        gicp_alignment.run();
        PointCloudRGB::Ptr aligned_cloud(new PointCloudRGB);
        gicp_alignment.getAlignedCloud(aligned_cloud);
        check(gicp_alignment.transform_exists_, "testRunWithCov_exists");
        const Eigen::Matrix4f T = gicp_alignment.getFineTransform();
        print_tf("testRunWithCov_run", T, gicp_alignment.transform_exists_);
        std::printf("testRunWithCov_sizes %zu %zu\n", sourceRGB->points.size(), targetRGB->points.size());
        gicp_alignment.iterate();
        check(gicp_alignment.transform_exists_, "testRunWithCov_iterate_exists");
        check(gicp_alignment.getFineTransform() == T * T, "testRunWithCov_iterate_composes");
        print_tf("testRunWithCov_iterate", gicp_alignment.getFineTransform(), gicp_alignment.transform_exists_);
        gicp_alignment.undo();
        PointCloudRGB::Ptr undone(new PointCloudRGB);
        gicp_alignment.getAlignedCloud(undone);
        check(same_xyz(*undone, *aligned_cloud), "testRunWithCov_undo");
    }
    {  // error paths (src/GICPAlignment.cpp:101-108, SURVEY 5 failure row): a good
       // run, then an empty source, then a source with fewer points than k = 20 -- each run must log
       // the failure and leave transform_exists_ and the fine transform untouched
        PointCloudRGB::Ptr sourceRGB(new PointCloudRGB(*sourceRGB0)), targetRGB(new PointCloudRGB(*targetRGB0));
        GICPAlignment g(targetRGB, sourceRGB, false);
        ros::Time::init();
        g.run();
        const Eigen::Matrix4f T_good = g.getFineTransform();
        check(g.transform_exists_, "errors_good_run_exists");
        PointCloudRGB::Ptr empty(new PointCloudRGB);
        g.setSourceCloud(empty);
        const int e0 = ros::error_count();
        g.run();
        check(ros::error_count() > e0, "errors_empty_source_logged");
        check(g.transform_exists_ && g.getFineTransform() == T_good, "errors_empty_source_untouched");
        PointCloudRGB::Ptr few(new PointCloudRGB);
        for (int i = 0; i < 10; ++i)
            few->push_back(sourceRGB0->points[static_cast<size_t>(i)]);
        g.setSourceCloud(few);
        const int e1 = ros::error_count();
        g.run();
        check(ros::error_count() > e1, "errors_too_few_points_logged");
        check(g.transform_exists_ && g.getFineTransform() == T_good, "errors_too_few_points_untouched");
        g.setTargetCloud(empty);
        g.setSourceCloud(sourceRGB);
        const int e2 = ros::error_count();
        g.run();
        check(ros::error_count() > e2, "errors_empty_target_logged");
        check(g.transform_exists_ && g.getFineTransform() == T_good, "errors_empty_target_untouched");
        std::printf("errors_logged %d\n", ros::error_count());
    }
    {  // the solver-failure path: a source 10 m off the target leaves fewer than 4
       // correspondences inside the gate -> PCL's estimateRigidTransformationBFGS throws, the
       // exception is caught in computeTransformation, and align() still writes
       // output = (previous * guess) * source.  So run() logs "no converge" and leaves fine_tf_, and
       // iterate() (src/GICPAlignment.cpp:116) overwrites aligned_cloud_ with the far source under T = I
        PointCloudRGB::Ptr sourceRGB(new PointCloudRGB(*sourceRGB0)), targetRGB(new PointCloudRGB(*targetRGB0));
        GICPAlignment g(targetRGB, sourceRGB, false);
        ros::Time::init();
        g.run();
        const Eigen::Matrix4f T_good = g.getFineTransform();
        check(g.transform_exists_, "solver_good_run_exists");
        PointCloudRGB::Ptr far(new PointCloudRGB);
        for (int i = 0; i < 30; ++i)
        {
            pcl::PointXYZRGB p = sourceRGB0->points[static_cast<size_t>(i) * 97];
            p.x += 10.f;
            far->push_back(p);
        }
        g.setSourceCloud(far);
        const int e0 = ros::error_count();
        g.run();
        check(ros::error_count() > e0, "solver_run_logged");
        check(g.transform_exists_ && g.getFineTransform() == T_good, "solver_run_untouched");
        const int e1 = ros::error_count();
        g.iterate();
        check(ros::error_count() > e1, "solver_iterate_logged");
        check(g.getFineTransform() == T_good, "solver_iterate_untouched");
        PointCloudRGB::Ptr aligned(new PointCloudRGB);
        g.getAlignedCloud(aligned);
        check(same_xyz(*aligned, *far), "solver_iterate_output_written");
    }
    {  // the Filter members either side of the path (adapter/Filter_mi355x.cpp)
        PointCloudRGB::Ptr src(new PointCloudRGB(*sourceRGB0));
        Filter f(0.25);
        PointCloudRGB::Ptr down(new PointCloudRGB);
        f.downsampleCloud(src, down);
        check(!down->points.empty() && down->points.size() < src->points.size(), "filter_downsample");
        std::printf("filter_downsample_count %zu\n", down->points.size());
        PointCloudRGB::Ptr diff(new PointCloudRGB), empty(new PointCloudRGB);
        Filter::removeFromCloud(src, src, 1e-6, diff);
        check(diff->points.empty(), "filter_difference_self_empty");
        Filter::removeFromCloud(src, empty, 1e-6, diff);
        check(diff->points.size() == src->points.size(), "filter_difference_empty_target_keeps_all");
    }
    std::printf("failures %d\n", g_fail);
    return g_fail ? 1 : 0;
}
