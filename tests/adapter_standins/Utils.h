/*
 * TEST INFRASTRUCTURE ONLY -- stand-in of the reference's include/Utils.h: the same class name
 * and the signatures of the members the adapter calls (/root/reference/include/Utils.h:122,151,
 * 175,182), over the layout-exact PCL / Eigen / ROS stand-ins of standin_deps.h.
 */
#pragma once

#include "standin_deps.h"

class Utils
{
    typedef pcl::PointCloud<pcl::PointXYZ> PointCloudXYZ;
    typedef pcl::PointCloud<pcl::PointXYZRGB> PointCloudRGB;

public:
    Utils() = delete;
    static bool isValidCloud(PointCloudRGB::Ptr cloud);
    static bool isValidTransform(Eigen::Matrix4f transform);
    static void cloudToROSMsg(PointCloudRGB::Ptr cloud, sensor_msgs::PointCloud2& cloud_msg,
                              const std::string& frameid = "world");
    static double computeCloudResolution(PointCloudRGB::Ptr cloud);
    static void printTransform(const Eigen::Matrix4f& transform);
};
