package ai.foremast.metrics.servlet;

import io.micrometer.core.instrument.binder.tomcat.TomcatMetrics;

import javax.servlet.ServletContext;
import javax.servlet.ServletContextEvent;
import javax.servlet.ServletContextListener;
import java.lang.reflect.Field;
import java.util.Collections;
import java.util.HashMap;
import java.util.Map;

/**
 * Binds the container's session metrics once the web application starts (the
 * reference 1.x starter's TomcatMetricsBinder role,
 * foremast-spring-boot-1x-k8s-metrics-starter/.../TomcatMetricsBinder.java):
 * on Tomcat the {@code org.apache.catalina.Context} behind the servlet
 * context is found by reflection (no compile-time catalina dependency) and
 * Micrometer's {@link TomcatMetrics} bound with its session {@code Manager}
 * -- the {@code tomcat_sessions_*} series the recording rules read.  On
 * another container (or {@code tomcatMetrics=false}) it binds the JMX-only
 * Tomcat meters (thread pools, global request processor) when present, or
 * nothing.  Context parameters are the module's settings.
 */
public class ForemastMetricsListener implements ServletContextListener {

    @Override
    public void contextInitialized(ServletContextEvent event) {
        ServletContext ctx = event.getServletContext();
        Map<String, String> s = new HashMap<>();
        for (String k : Collections.list(ctx.getInitParameterNames())) {
            s.put(k, ctx.getInitParameter(k));
        }
        ForemastMetrics metrics = ForemastMetrics.shared(s);
        if ("false".equals(s.get("tomcatMetrics"))) {
            return;
        }
        try {
            Class.forName("org.apache.catalina.Manager", false, ctx.getClass().getClassLoader());
        } catch (ClassNotFoundException | LinkageError e) {
            return;                                   // not Tomcat
        }
        new TomcatMetrics(catalinaManager(ctx), Collections.emptyList()).bindTo(metrics.registry());
    }

    /** The session manager of Tomcat's Context behind the facade, or null. */
    static org.apache.catalina.Manager catalinaManager(ServletContext ctx) {
        try {
            Object appCtx = field(ctx, "context");          // ApplicationContextFacade -> ApplicationContext
            Object std = appCtx == null ? null : field(appCtx, "context");   // -> StandardContext
            if (std instanceof org.apache.catalina.Context) {
                return ((org.apache.catalina.Context) std).getManager();
            }
        } catch (ReflectiveOperationException | RuntimeException e) {
            // an unexpected facade: session meters stay unbound
        }
        return null;
    }

    private static Object field(Object o, String name) throws ReflectiveOperationException {
        for (Class<?> c = o.getClass(); c != null; c = c.getSuperclass()) {
            try {
                Field f = c.getDeclaredField(name);
                f.setAccessible(true);
                return f.get(o);
            } catch (NoSuchFieldException e) {
                // up the hierarchy
            }
        }
        return null;
    }

    @Override
    public void contextDestroyed(ServletContextEvent event) {
    }
}
