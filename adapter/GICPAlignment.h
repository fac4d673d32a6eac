/*
 * adapter/GICPAlignment.h -- drop-in header for the reference package
 * (replaces /root/reference/include/GICPAlignment.h).
 *
 * Public surface: identical to the reference (include/GICPAlignment.h:32-145) so that
 * LeicaStateMachine (src/LeicaStateMachine.cpp:149-153), the ROS node and
 * test/test_gicp_alignment.cpp compile unchanged.  Private section: the PCL GICP member
 * (include/GICPAlignment.h:153) is replaced by a handle of the MI355X engine (libmgicp.so,
 * include/mi355x_gicp.h).  See INTEGRATION.md.
 */
#pragma once
#ifndef _GICP_ALIGNMENT_H
#define _GICP_ALIGNMENT_H

#include <Utils.h>
#include <mi355x_gicp.h>

class GICPAlignment
{
    typedef pcl::PointCloud<pcl::PointXYZ> PointCloudXYZ;
    typedef pcl::PointCloud<pcl::PointXYZRGB> PointCloudRGB;

public:
    // NB: target first, as in the reference
    GICPAlignment(PointCloudRGB::Ptr target_cloud, PointCloudRGB::Ptr source_cloud, bool use_covariances);
    ~GICPAlignment();

    bool transform_exists_;

    void run();
    void iterate();
    void undo();
    Eigen::Matrix4f getFineTransform();
    void getAlignedCloud(PointCloudRGB::Ptr aligned_cloud);
    void getAlignedCloudROSMsg(sensor_msgs::PointCloud2& aligned_cloud_msg);
    void applyTFtoCloud(PointCloudRGB::Ptr cloud);
    void setSourceCloud(PointCloudRGB::Ptr source_cloud);
    void setTargetCloud(PointCloudRGB::Ptr target_cloud);
    void setMaxIterations(int iterations);
    void setTfEpsilon(double tf_epsilon);
    void setMaxCorrespondenceDistance(int max_corresp_distance);  // int: doubles truncate (kept)
    void setRANSACOutlierTh(int ransac_threshold);                // int: doubles truncate (kept)

private:
    GICPAlignment(const GICPAlignment&) = delete;
    GICPAlignment& operator=(const GICPAlignment&) = delete;

    bool covariances_;
    mgicp_ctx* engine_;        // replaces pcl::GeneralizedIterativeClosestPoint<XYZRGB,XYZRGB>
    mgicp_params engine_params_;
    double ransac_outlier_th_; // kept for the setter; GICP never used it

    Eigen::Matrix4f fine_tf_;
    int max_iter_;
    double tf_epsilon_;
    double max_corresp_distance_;

    PointCloudRGB::Ptr target_cloud_;
    PointCloudRGB::Ptr source_cloud_;
    PointCloudRGB::Ptr aligned_cloud_;
    PointCloudRGB::Ptr backup_cloud_;

    void configParameters();
    void fineAlignment();
    void getCovariances(PointCloudRGB::Ptr cloud);
    void applyCovariances();
    void iterateFineAlignment(PointCloudRGB::Ptr cloud);
    void backUp(PointCloudRGB::Ptr cloud);
    bool alignOnce(PointCloudRGB::Ptr output, Eigen::Matrix4f& T);
    void logFitness(const Eigen::Matrix4f& T);
};

#endif
