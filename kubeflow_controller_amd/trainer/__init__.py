"""trainer"""
