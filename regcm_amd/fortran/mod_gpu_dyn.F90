!
! mod_gpu_dyn -- Fortran 2003 ISO_C_BINDING shim over the rcmdyn C-ABI (include/rcmdyn.h).
!
! This is the module a RegCM 4.7 host links to run the dynamical-core step on MI355X
! instead of `call tend` / `call bdyval` (Main/mod_regcm_interface.F90:189,208).  Arrays are
! passed with their Fortran bounds exactly as getmem* allocated them (j fastest), so the
! host keeps its own layout and never sees device memory.  See INTEGRATION.md.
!
module mod_gpu_dyn
  use iso_c_binding
  implicit none
  private

  integer, parameter, public :: rcmdyn_abi_version = 6
  integer, parameter, public :: rcmdyn_maxkz = 64, rcmdyn_maxsplit = 4

  ! field ids (enum rcmdyn_field)
  integer(c_int32_t), parameter, public :: &
    f_atm1_u = 0, f_atm1_v = 1, f_atm1_t = 2, f_atm1_qv = 3, f_atm1_qc = 4, &
    f_atm2_u = 5, f_atm2_v = 6, f_atm2_t = 7, f_atm2_qv = 8, f_atm2_qc = 9, &
    f_psa = 10, f_psb = 11, f_dstor = 12, f_hstor = 13, &
    f_msfx = 14, f_msfd = 15, f_coriol = 16, f_ht = 17, &
    f_xub_b0 = 18, f_xub_bt = 19, f_xvb_b0 = 20, f_xvb_bt = 21, f_xtb_b0 = 22, &
    f_xtb_bt = 23, f_xqb_b0 = 24, f_xqb_bt = 25, f_xpsb_b0 = 26, f_xpsb_bt = 27, &
    f_psc = 28, f_pten = 29, f_psdota = 30, f_tten = 31, f_uten = 32, f_vten = 33, &
    f_qvten = 34, f_qcten = 35, f_omega = 36, f_qdot = 37, f_xkc = 38, f_phi = 39, &
    f_atm1_pp = 40, f_atm2_pp = 41, f_atm1_w = 42, f_atm2_w = 43, &
    f_xppb_b0 = 44, f_xppb_bt = 45, f_xwwb_b0 = 46, f_xwwb_bt = 47, &
    f_atm0_ps = 48, f_atm0_pr = 49, f_atm0_t = 50, f_atm0_rho = 51, f_atm0_z = 52, &
    f_atm0_pf = 53, f_atm0_rhof = 54, f_atm0_zf = 55, f_dpsdxm = 56, f_dpsdym = 57, &
    f_dprddx = 58, f_dprddy = 59, f_ef = 60, f_ddx = 61, f_ddy = 62, f_dmdx = 63, &
    f_dmdy = 64, f_ex = 65, f_crx = 66, f_cry = 67, &
    ! physics coupling seam: pc_physic tendencies (put) and the mkslice export (get)
    f_tphy = 68, f_qvphy = 69, f_qcphy = 70, f_uphy = 71, f_vphy = 72, f_ppphy = 73, f_wphy = 74, &
    f_atms_ubx3d = 75, f_atms_vbx3d = 76, f_atms_ubd3d = 77, f_atms_vbd3d = 78, f_atms_tb3d = 79, &
    f_atms_qvb3d = 80, f_atms_qcb3d = 81, f_atms_tv3d = 82, f_atms_pb3d = 83, f_atms_pf3d = 84, &
    f_atms_ps2d = 85, f_atms_rhox2d = 86, f_atms_th3d = 87, f_atms_rhob3d = 88, f_atms_tp3d = 89, &
    f_atms_wpx3d = 90, f_atms_wb3d = 91, f_atms_zq = 92, f_atms_za = 93, f_atms_dzq = 94, &
    f_atms_qsb3d = 95, f_atms_rhb3d = 96, &
    ! device bdyin: the next ICBC record as read_icbc returns it; NH atm0%psdot
    f_xub_b1 = 97, f_xvb_b1 = 98, f_xtb_b1 = 99, f_xqb_b1 = 100, f_xpsb_b1 = 101, &
    f_xppb_b1 = 102, f_xwwb_b1 = 103, f_atm0_psdot = 104, &
    f_atm1_tke = 105, f_atm2_tke = 106, f_tkephy = 107, f_kpbl = 108, &
    ! nqx = 5 (ipptls >= 2): atm1/atm2 qx(:,:,:,iqi|iqr|iqs), their qxphy, the qxb3d export
    f_atm1_qi = 109, f_atm1_qr = 110, f_atm1_qs = 111, f_atm2_qi = 112, f_atm2_qr = 113, &
    f_atm2_qs = 114, f_qiphy = 115, f_qrphy = 116, f_qsphy = 117, &
    f_atms_qxb3d_qi = 118, f_atms_qxb3d_qr = 119, f_atms_qxb3d_qs = 120

  type, bind(c), public :: rcmdyn_config
    integer(c_int32_t) :: abi_version
    integer(c_int32_t) :: jx, iy, kz
    integer(c_int32_t) :: nproc_j, nproc_i
    integer(c_int32_t) :: tile_first, tile_count
    integer(c_int32_t) :: idynamic, iboudy, idiffu, ipgf, nsplit, nspgx, nspgd
    integer(c_int32_t) :: diffu_hgtf, upstream_mode, stability_enhance, present_qc
    real(c_double) :: ds, dtsec, ptop, gnu1, gnu2, uoffc, t_extrema, q_rel_extrema
    real(c_double) :: ckh, adyndif, high_nudge, medium_nudge, low_nudge
    real(c_double) :: bdy_nm, bdy_dm, dtbdys
    real(c_double) :: sigma(rcmdyn_maxkz+1)
    real(c_double) :: zmatx(rcmdyn_maxkz,rcmdyn_maxsplit)   ! zmatx(k,l)
    real(c_double) :: zmatxr(rcmdyn_maxkz,rcmdyn_maxsplit)  ! zmatxr(l,k) stored (k,l)
    real(c_double) :: am(rcmdyn_maxkz,rcmdyn_maxsplit)      ! am(k,l)
    real(c_double) :: tau(rcmdyn_maxkz,rcmdyn_maxsplit)     ! tau(l,k) stored (k,l)
    real(c_double) :: varpa1(rcmdyn_maxkz+1,rcmdyn_maxsplit)! varpa1(l,k) stored (k,l)
    real(c_double) :: an(rcmdyn_maxsplit), hbar(rcmdyn_maxsplit)
    real(c_double) :: aam(rcmdyn_maxsplit), dtau(rcmdyn_maxsplit)
    real(c_double) :: sigmah(rcmdyn_maxkz+1)
    real(c_double) :: pd
    integer(c_int32_t) :: comm_rank, comm_size, device
    integer(c_int8_t) :: comm_unique_id(128)
    ! non-hydrostatic core (nonhydroparam, init_sound outputs)
    integer(c_int32_t) :: ifupr, ifrayd, rayndamp, nh_reserved
    real(c_double) :: nhbet, nhxkd, rayalpha0, rayhd, nh_dtsmax, nh_xmsf
    ! cldparam rhmin, rhmax (mkslice rhb3d clamps)
    real(c_double) :: rhmin, rhmax
    ! physicsparam isladvec, iqmsl (semi-Lagrangian moisture advection)
    integer(c_int32_t) :: isladvec, iqmsl
    ! physicsparam ibltyp (2 = UW PBL TKE in the dyn step), uwparam iuwvadv, nuk, tkemin (uwtkemin)
    integer(c_int32_t) :: ibltyp, iuwvadv
    real(c_double) :: nuk, tkemin
    ! ABI 6: physicsparam ipptls and the nqx param sets from it (2, or 5 for ipptls >= 2);
    ! i_band (1: tropical band, hydrostatic core), i_crm, ichem (refused if set)
    integer(c_int32_t) :: ipptls, nqx
    integer(c_int32_t) :: i_band, i_crm, ichem
  end type rcmdyn_config

  interface
    integer(c_int) function rcmdyn_create(cfg, h) bind(c, name='rcmdyn_create')
      import :: c_int, c_ptr, rcmdyn_config
      type(rcmdyn_config), intent(in) :: cfg
      type(c_ptr), intent(out) :: h
    end function
    integer(c_int) function rcmdyn_destroy(h) bind(c, name='rcmdyn_destroy')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
    end function
    type(c_ptr) function rcmdyn_last_error(h) bind(c, name='rcmdyn_last_error')
      import :: c_ptr
      type(c_ptr), value :: h
    end function
    integer(c_int) function rcmdyn_put(h, f, src, j1, j2, i1, i2, k1, k2) bind(c, name='rcmdyn_put')
      import :: c_int, c_ptr, c_int32_t, c_double
      type(c_ptr), value :: h
      integer(c_int32_t), value :: f, j1, j2, i1, i2, k1, k2
      real(c_double), intent(in) :: src(*)
    end function
    integer(c_int) function rcmdyn_get(h, f, dst, j1, j2, i1, i2, k1, k2) bind(c, name='rcmdyn_get')
      import :: c_int, c_ptr, c_int32_t, c_double
      type(c_ptr), value :: h
      integer(c_int32_t), value :: f, j1, j2, i1, i2, k1, k2
      real(c_double), intent(out) :: dst(*)
    end function
    integer(c_int) function rcmdyn_set_time(h, lcount, dt, xbctime) bind(c, name='rcmdyn_set_time')
      import :: c_int, c_ptr, c_int64_t, c_double
      type(c_ptr), value :: h
      integer(c_int64_t), value :: lcount
      real(c_double), value :: dt, xbctime
    end function
    integer(c_int) function rcmdyn_get_time(h, lcount, dt, xbctime) bind(c, name='rcmdyn_get_time')
      import :: c_int, c_ptr, c_int64_t, c_double
      type(c_ptr), value :: h
      integer(c_int64_t), intent(out) :: lcount
      real(c_double), intent(out) :: dt, xbctime
    end function
    integer(c_int) function rcmdyn_tend(h) bind(c, name='rcmdyn_tend')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
    end function
    integer(c_int) function rcmdyn_tend_pre_physics(h) bind(c, name='rcmdyn_tend_pre_physics')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
    end function
    integer(c_int) function rcmdyn_tend_post_physics(h) bind(c, name='rcmdyn_tend_post_physics')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
    end function
    integer(c_int) function rcmdyn_bdyin(h) bind(c, name='rcmdyn_bdyin')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
    end function
    integer(c_int) function rcmdyn_bdyval(h) bind(c, name='rcmdyn_bdyval')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
    end function
    integer(c_int) function rcmdyn_step(h, n) bind(c, name='rcmdyn_step')
      import :: c_int, c_ptr, c_int32_t
      type(c_ptr), value :: h
      integer(c_int32_t), value :: n
    end function
    ! the 3-hourly report sums (sumall/maxall over the job): ptntot, pt2tot, NH max CFL
    integer(c_int) function rcmdyn_reductions(h, out) bind(c, name='rcmdyn_reductions')
      import :: c_int, c_ptr, c_double
      type(c_ptr), value :: h
      real(c_double), intent(out) :: out(3)
    end function
    integer(c_int) function rcmdyn_diagnostics(h, out) bind(c, name='rcmdyn_diagnostics')
      import :: c_int, c_ptr, c_double
      type(c_ptr), value :: h
      real(c_double), intent(out) :: out(4)
    end function
    integer(c_int) function rcmdyn_comm_unique_id(out) bind(c, name='rcmdyn_comm_unique_id')
      import :: c_int, c_int8_t
      integer(c_int8_t), intent(out) :: out(128)
    end function
    ! waits for the device and reports any failed step; COLLECTIVE in RCCL mode (every rank
    ! calls it, as every rank calls rcmdyn_step)
    integer(c_int) function rcmdyn_synchronize(h) bind(c, name='rcmdyn_synchronize')
      import :: c_int, c_ptr
      type(c_ptr), value :: h
    end function
    ! set_nproc (Main/mpplib/mod_mppparam.F90:1053-1371), host-only: cpus = (cpus_j, cpus_i)
    integer(c_int) function rcmdyn_set_nproc(nproc, jx, iy, cpus) bind(c, name='rcmdyn_set_nproc')
      import :: c_int, c_int32_t
      integer(c_int32_t), value :: nproc, jx, iy
      integer(c_int32_t), intent(out) :: cpus(2)
    end function
    ! ext = (jde1,jde2,ide1,ide2,jce1,jce2,ice1,ice2), bdy = (left,right,bottom,top), host-only
    integer(c_int) function rcmdyn_tile_extent(jx, iy, nproc_j, nproc_i, tile, ext, bdy) &
        bind(c, name='rcmdyn_tile_extent')
      import :: c_int, c_int32_t
      integer(c_int32_t), value :: jx, iy, nproc_j, nproc_i, tile
      integer(c_int32_t), intent(out) :: ext(8), bdy(4)
    end function
    ! the same for cfg's grid and decomposition with its periodic directions (i_band: j,
    ! i_crm: i), as the engine's tiles are cut; host-only
    integer(c_int) function rcmdyn_tile_extent_cfg(cfg, tile, ext, bdy) bind(c, name='rcmdyn_tile_extent_cfg')
      import :: c_int, c_int32_t, rcmdyn_config
      type(rcmdyn_config), intent(in) :: cfg
      integer(c_int32_t), value :: tile
      integer(c_int32_t), intent(out) :: ext(8), bdy(4)
    end function
    ! the communication calls of one rank (7 int64 per record), host-only
    integer(c_int) function rcmdyn_exchange_plan(cfg, nsteps, ops, cap, count) bind(c, name='rcmdyn_exchange_plan')
      import :: c_int, c_int32_t, c_int64_t, rcmdyn_config
      type(rcmdyn_config), intent(in) :: cfg
      integer(c_int32_t), value :: nsteps
      integer(c_int64_t), intent(out) :: ops(*)
      integer(c_int64_t), value :: cap
      integer(c_int64_t), intent(out) :: count
    end function
    ! per tile, the points of the update kernels that run beside the prologue exchange
    integer(c_int) function rcmdyn_overlap_shares(cfg, out, cap) bind(c, name='rcmdyn_overlap_shares')
      import :: c_int, c_int32_t, rcmdyn_config
      type(rcmdyn_config), intent(in) :: cfg
      integer(c_int32_t), intent(out) :: out(*)
      integer(c_int32_t), value :: cap
    end function
    ! the HIP runtime and librccl the engine is bound to (a NUL-terminated string)
    integer(c_int) function rcmdyn_runtime_info(buf, len) bind(c, name='rcmdyn_runtime_info')
      import :: c_int, c_char, c_int32_t
      character(kind=c_char), intent(out) :: buf(*)
      integer(c_int32_t), value :: len
    end function
    ! average device ms per step of the last rcmdyn_step call
    integer(c_int) function rcmdyn_last_step_ms(h, ms) bind(c, name='rcmdyn_last_step_ms')
      import :: c_int, c_ptr, c_double
      type(c_ptr), value :: h
      real(c_double), intent(out) :: ms
    end function
    ! the per-point tendency diagnostics (f_tten .. f_xkc) on (1) or off (0, the default)
    integer(c_int) function rcmdyn_set_diagnostics(h, on) bind(c, name='rcmdyn_set_diagnostics')
      import :: c_int, c_ptr, c_int32_t
      type(c_ptr), value :: h
      integer(c_int32_t), value :: on
    end function
    ! per-kernel device time over nsteps eager steps (names: 48 characters per kernel)
    integer(c_int) function rcmdyn_kernel_times(h, nsteps, cap, names, launches, avg_ms, count) &
        bind(c, name='rcmdyn_kernel_times')
      import :: c_int, c_ptr, c_int32_t, c_char, c_double
      type(c_ptr), value :: h
      integer(c_int32_t), value :: nsteps, cap
      character(kind=c_char), intent(out) :: names(*)
      integer(c_int32_t), intent(out) :: launches(*)
      real(c_double), intent(out) :: avg_ms(*)
      integer(c_int32_t), intent(out) :: count
    end function
  end interface

  public :: rcmdyn_create, rcmdyn_destroy, rcmdyn_put, rcmdyn_get, rcmdyn_set_time
  public :: rcmdyn_get_time, rcmdyn_tend, rcmdyn_bdyval, rcmdyn_step, rcmdyn_diagnostics, rcmdyn_reductions
  public :: rcmdyn_tend_pre_physics, rcmdyn_tend_post_physics, rcmdyn_bdyin, rcmdyn_last_error
  public :: rcmdyn_synchronize, rcmdyn_set_nproc, rcmdyn_tile_extent, rcmdyn_tile_extent_cfg, rcmdyn_exchange_plan
  public :: rcmdyn_overlap_shares, rcmdyn_runtime_info, rcmdyn_last_step_ms, rcmdyn_set_diagnostics
  public :: rcmdyn_kernel_times
  public :: rcmdyn_comm_unique_id, gpu_dyn_check, gpu_put3d, gpu_get3d, gpu_put2d, gpu_get2d

  contains

  ! Abort like the reference's fatal() (Share/mod_message.F90:90-103) on any engine error.
  subroutine gpu_dyn_check(h, ierr, where)
    type(c_ptr), intent(in) :: h
    integer(c_int), intent(in) :: ierr
    character(len=*), intent(in) :: where
    character(kind=c_char), pointer :: msg(:)
    integer :: n
    if ( ierr == 0 ) return
    call c_f_pointer(rcmdyn_last_error(h), msg, [1024])
    n = 0
    do while ( n < 1024 )
      if ( msg(n+1) == c_null_char ) exit
      n = n + 1
    end do
    write(0,*) 'mod_gpu_dyn: ', where, ': ', msg(1:n)
    error stop 1
  end subroutine gpu_dyn_check

  ! Put/get a pointer array allocated as a(j1:j2,i1:i2,k1:k2) by getmem3d: pointer
  ! dummies keep the host's lower bounds, which the C-ABI takes as global indices.
  subroutine gpu_put3d(h, f, a)
    type(c_ptr), intent(in) :: h
    integer(c_int32_t), intent(in) :: f
    real(c_double), pointer, contiguous, intent(in) :: a(:,:,:)
    call gpu_dyn_check(h, rcmdyn_put(h, f, a, lbound(a,1), ubound(a,1), lbound(a,2), &
         ubound(a,2), lbound(a,3), ubound(a,3)), 'put3d')
  end subroutine gpu_put3d
  subroutine gpu_get3d(h, f, a)
    type(c_ptr), intent(in) :: h
    integer(c_int32_t), intent(in) :: f
    real(c_double), pointer, contiguous, intent(in) :: a(:,:,:)
    call gpu_dyn_check(h, rcmdyn_get(h, f, a, lbound(a,1), ubound(a,1), lbound(a,2), &
         ubound(a,2), lbound(a,3), ubound(a,3)), 'get3d')
  end subroutine gpu_get3d
  subroutine gpu_put2d(h, f, a)
    type(c_ptr), intent(in) :: h
    integer(c_int32_t), intent(in) :: f
    real(c_double), pointer, contiguous, intent(in) :: a(:,:)
    call gpu_dyn_check(h, rcmdyn_put(h, f, a, lbound(a,1), ubound(a,1), lbound(a,2), &
         ubound(a,2), 1, 1), 'put2d')
  end subroutine gpu_put2d
  subroutine gpu_get2d(h, f, a)
    type(c_ptr), intent(in) :: h
    integer(c_int32_t), intent(in) :: f
    real(c_double), pointer, contiguous, intent(in) :: a(:,:)
    call gpu_dyn_check(h, rcmdyn_get(h, f, a, lbound(a,1), ubound(a,1), lbound(a,2), &
         ubound(a,2), 1, 1), 'get2d')
  end subroutine gpu_get2d

end module mod_gpu_dyn
